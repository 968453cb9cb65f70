// mfma4_bench.hip — v_mfma_f32_4x4x1_16b_f32 on gfx950: (1) operand / result lane map checked with
// exact integer data, (2) back-to-back issue cost per instruction with 1 and 2 waves per SIMD and
// 1 / 4 independent accumulators, next to v_mfma_f32_16x16x4_f32 for scale.
// Hypothesis checked: lane l = 4b + j holds A_b[m = j] and B_b[n = j] of block b = l / 4; result
// register i of lane 4b + j = D_b[m = i][n = j] = Σ_k A_b[i] B_b[j] (K = 1 per instruction).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void layout(const float *A, const float *B, float *D) {
    const int l = threadIdx.x;
    f4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(A[64 + l], B[64 + l], c, 0, 0, 0);   // second k
    for (int i = 0; i < 4; ++i) D[l * 4 + i] = c[i];
}

template <int NACC, bool BIG>
__global__ void rate(float *out, int iters, float a0, float b0) {
    f4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
    float a = a0 + threadIdx.x, b = b0 - threadIdx.x;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) {
            if (BIG) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
            else acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
        }
    }
    const long long t1 = clock64();
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[1 << 20] = (float)(t1 - t0) / (float)(iters * NACC);
}

int main() {
    float hA[128], hB[128], hD[256];
    for (int i = 0; i < 128; ++i) { hA[i] = (float)(rand() % 17 - 8); hB[i] = (float)(rand() % 13 - 6); }
    float *dA, *dB, *dD, *dO;
    hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 1024); hipMalloc(&dO, ((1 << 20) + 64) * 4);
    hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) {
            const int b = l / 4, j = l % 4;
            const float ref = hA[4 * b + i] * hB[4 * b + j] + hA[64 + 4 * b + i] * hB[64 + 4 * b + j];
            if (hD[l * 4 + i] != ref) ++bad;
        }
    printf("mfma 4x4x1_16b layout hypothesis: %d mismatches of 256\n", bad);
    const int iters = 4096;
    auto run = [&](const char *name, void (*kf)(float *, int, float, float), int threads) {
        hipLaunchKernelGGL(kf, dim3(1), dim3(threads), 0, 0, dO, iters, 1.0f, 2.0f);
        hipLaunchKernelGGL(kf, dim3(1), dim3(threads), 0, 0, dO, iters, 1.0f, 2.0f);
        hipDeviceSynchronize();
        float cyc;
        hipMemcpy(&cyc, dO + (1 << 20), 4, hipMemcpyDeviceToHost);
        printf("%-28s threads %4d: %.2f clock64 ticks per instruction per wave\n", name, threads, cyc);
    };
    run("4x4x1_16b, 1 acc", rate<1, false>, 256);
    run("4x4x1_16b, 4 acc", rate<4, false>, 256);
    run("4x4x1_16b, 4 acc", rate<4, false>, 512);
    run("4x4x1_16b, 8 acc", rate<8, false>, 256);
    run("16x16x4, 1 acc", rate<1, true>, 256);
    run("16x16x4, 4 acc", rate<4, true>, 256);
    run("16x16x4, 4 acc", rate<4, true>, 512);
    return bad != 0;
}
