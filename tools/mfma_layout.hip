#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef float f4 __attribute__((ext_vector_type(4)));
// D[i][j] = sum_k A[i][k] * B[k][j], 16x16x4; check lane layout assumptions
__global__ void k(const float* A, const float* B, float* D) {
    int l = threadIdx.x;
    float a = A[(l % 16) * 4 + l / 16];        // A[i=l%16][k=l/16]
    float b = B[(l / 16) * 16 + l % 16];       // B[k=l/16][j=l%16]
    f4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + l % 16] = c[r];   // D[i=4(l/16)+r][j=l%16]
}
int main() {
    float hA[64], hB[64], hD[256], ref[256];
    for (int i = 0; i < 64; ++i) { hA[i] = (float)(rand() % 17) - 8; hB[i] = (float)(rand() % 13) - 6; }
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { float s = 0; for (int kk = 0; kk < 4; ++kk) s += hA[i * 4 + kk] * hB[kk * 16 + j]; ref[i * 16 + j] = s; }
    float *dA, *dB, *dD;
    hipMalloc(&dA, 256); hipMalloc(&dB, 256); hipMalloc(&dD, 1024);
    hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 256; ++i) if (fabsf(hD[i] - ref[i]) > 1e-4) ++bad;
    printf("mfma 16x16x4f32 layout check: %d mismatches of 256\n", bad);
    return bad != 0;
}
