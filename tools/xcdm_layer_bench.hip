// xcdm_layer_bench.hip — cycles per call of the many-row XCD kernel's MFMA layers (mlayer_any of
// fatchord_xcdm.hip, compiled in from the kernel source itself) on every CU at once, one
// workgroup of kMThreads per CU as in the kernel: A operands in registers, the staged slice and
// the partials in LDS.  Prints s_memtime cycles per call (MFMAs + partial-sum epilogue + LDS wait).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I include -I wavernn_amd/csrc \
//       tools/xcdm_layer_bench.hip -o tools/xcdm_layer_bench
#include "../wavernn_amd/csrc/fatchord_xcdm.hip"

#include <cstdio>

namespace wrnn {

template <int NQ, int S0, int NS>
__global__ __launch_bounds__(kMThreads, 1) void layer_bench(const float *W, float *out, int iters) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int kStgQ = xcdm_big(NQ) ? kMQuadMax : NQ;
    float *stg = smem + wave * kStgQ * kMStg;
    float *P = smem + kMWaves * kStgQ * kMStg;
    for (int i = lane; i < kStgQ * kMStg; i += 64) stg[i] = W[(i * 7 + wave) & 4095] * 0.5f;
    float A[kMSets][kMJ];
#pragma unroll
    for (int s = 0; s < kMSets; ++s)
#pragma unroll
        for (int j = 0; j < kMJ; ++j) A[s][j] = W[((s * kMJ + j) * 64 + lane) & 4095];
    __syncthreads();
    long long t0 = 0;
    for (int it = 0; it < iters; ++it) {
        if (it == 1) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            t0 = __builtin_amdgcn_s_memtime();
        }
        mlayer_any<NQ, S0, NS>(A, stg, P, lane, wave);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    float s = 0.0f;
    for (int i = tid; i < NS * 16 * 4 * NQ * kMWaves; i += kMThreads) s += P[i];
    out[blockIdx.x * kMThreads + tid] = s;
    if (tid == 0) out[(1 << 20) + blockIdx.x] = (float)(t1 - t0) / (float)(iters - 1);
}

}  // namespace wrnn

using namespace wrnn;

template <int NQ, int S0, int NS>
static void run(const char *name, const float *dW, float *dO, float *h) {
    constexpr int kStgQ = xcdm_big(NQ) ? kMQuadMax : NQ;
    const size_t lds = (kMWaves * kStgQ * kMStg + 3 * 16 * 4 * kMQuadMax * kMWaves) * sizeof(float);
    hipFuncSetAttribute((const void *)layer_bench<NQ, S0, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((layer_bench<NQ, S0, NS>), dim3(256), dim3(kMThreads), lds, 0, dW, dO, 65);
    hipDeviceSynchronize();
    hipMemcpy(h, dO + (1 << 20), 256 * sizeof(float), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += h[i];
    m /= 256;
    const int mf = NS * kMJ * (xcdm_big(NQ) ? 1 : NQ);
    printf("NQ %d %-14s %5.0f cycles per call  (%3d MFMAs per wave: %5.1f cycles each)\n", NQ, name, m, mf, m / mf);
}

int main() {
    float *dW, *dO, h[256], hw[4096];
    for (int i = 0; i < 4096; ++i) hw[i] = (float)((i * 37) % 101) / 101.0f - 0.5f;
    hipMalloc(&dW, 4096 * sizeof(float));
    hipMalloc(&dO, ((1 << 20) + 256) * sizeof(float));
    hipMemcpy(dW, hw, sizeof(hw), hipMemcpyHostToDevice);
    run<1, MS_IH2, 3>("ih2 (AGPR)", dW, dO, h);
    run<1, MS_HH1, 3>("hh1 (VGPR)", dW, dO, h);
    run<1, MS_FC1, 1>("fc1 (AGPR)", dW, dO, h);
    run<2, MS_IH2, 3>("ih2 (AGPR)", dW, dO, h);
    run<2, MS_FC1, 1>("fc1 (AGPR)", dW, dO, h);
    run<3, MS_IH2, 3>("ih2 (AGPR)", dW, dO, h);
    run<4, MS_IH2, 3>("ih2 (AGPR)", dW, dO, h);
    run<4, MS_HH1, 3>("hh1 (VGPR)", dW, dO, h);
    run<4, MS_FC1, 1>("fc1 (AGPR)", dW, dO, h);
    return 0;
}
