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
    for (int i = tid; i < NS * xcdm_pset(NQ); i += kMThreads) s += P[i];
    out[blockIdx.x * kMThreads + tid] = s;
    if (tid == 0) out[(1 << 20) + blockIdx.x] = (float)(t1 - t0) / (float)(iters - 1);
}

// the MFMA stream alone: 3 sets × 32 columns, NC chains per set, B from registers (no LDS) —
// kMode 0: one B register for all; 1: B[j] per column
template <int NC, int kMode>
__global__ __launch_bounds__(kMThreads, 1) void stream_bench(const float *W, float *out, int iters) {
    const int tid = threadIdx.x, lane = tid & 63;
    float A[kMSets][kMJ];
#pragma unroll
    for (int s = 0; s < kMSets; ++s)
#pragma unroll
        for (int j = 0; j < kMJ; ++j) A[s][j] = W[((s * kMJ + j) * 64 + lane) & 4095];
    float B[kMJ];
#pragma unroll
    for (int j = 0; j < kMJ; ++j) B[j] = W[(j * 64 + lane + 7) & 4095];
    long long t0 = 0;
    f4v tot = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        if (it == 1) t0 = __builtin_amdgcn_s_memtime();
        f4v acc[3][NC];
#pragma unroll
        for (int j = 0; j < kMJ; ++j)
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                const float b = kMode == 0 ? B[0] : B[j];
                if (j < NC) mfma_first<true>(acc[s][j % NC], A[s][j], b);
                else mfma_acc<true>(acc[s][j % NC], A[s][j], b);
            }
        mfma_drain_begin();
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) {
                mfma_tie(acc[s][cc]);
                tot += acc[s][cc];
            }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * kMThreads + tid] = tot.x + tot.y + tot.z + tot.w;
    if (tid == 0) out[(1 << 20) + blockIdx.x] = (float)(t1 - t0) / (float)(iters - 1);
}

// mlayer variants (NQ = 1): kDepth = B chunks in flight (2 = the kernel's double buffer, 8 = all
// of them read up front); kEpi = 0 no partials epilogue, 1 the kernel's mput
template <int NS, int NC, int kDepth, int kEpi>
__device__ __forceinline__ void mlayer_v(const float (&A)[kMSets][kMJ], const float *stg, float *P, int lane, int wave) {
    const int j4 = lane & 3, sp = lane >> 4;
    f4v acc[NS][NC];
    f4v b[kDepth];
#pragma unroll
    for (int d = 0; d < kDepth - 1; ++d) b[d] = lds4(stg + mstg_at(j4, kMJ * sp + 4 * d));
#pragma unroll
    for (int jc = 0; jc < kMJ / 4; ++jc) {
        if (jc + kDepth - 1 < kMJ / 4) b[(jc + kDepth - 1) % kDepth] = lds4(stg + mstg_at(j4, kMJ * sp + 4 * (jc + kDepth - 1)));
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * jc + jj;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                if (j < NC) mfma_first<true>(acc[s][j % NC], A[s][j], b[jc % kDepth][jj]);
                else mfma_acc<true>(acc[s][j % NC], A[s][j], b[jc % kDepth][jj]);
            }
        }
    }
    mfma_drain_begin();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) mfma_tie(acc[s][cc]);
    if (kEpi == 1) mput<1, NS, NC>(acc, P, 0, lane, wave);
    else if (kEpi == 2) {
        // unreduced k-slices: P[wave][set][row][n][sp], row stride 4·NR + 4 (conflict-free)
        constexpr int NR = 4, S = 4 * NR + 4;
        const int g = (lane >> 2) & 3, n = lane & 3, sp = lane >> 4;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            f4v d = acc[s][0];
#pragma unroll
            for (int cc = 1; cc < NC; ++cc) d += acc[s][cc];
            float *p = P + (wave * NS + s) * 16 * S + 4 * g * S + 4 * n + sp;
            p[0] = d.x;
            p[S] = d.y;
            p[2 * S] = d.z;
            p[3 * S] = d.w;
        }
    } else {
        f4v d = acc[0][0];
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) d += acc[s][cc];
        if (lane == 0) P[wave] = d.x + d.y + d.z + d.w;
    }
}

template <int NS, int NC, int kDepth, int kEpi>
__global__ __launch_bounds__(kMThreads, 1) void variant_bench(const float *W, float *out, int iters) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    float *stg = smem + wave * kMStg;
    float *P = smem + kMWaves * kMStg;
    for (int i = lane; i < kMStg; i += 64) stg[i] = W[(i * 7 + wave) & 4095] * 0.5f;
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
        mlayer_v<NS, NC, kDepth, kEpi>(A, stg, P, lane, wave);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    float s = 0.0f;
    for (int i = tid; i < NS * 16 * 4 * kMWaves; i += kMThreads) s += P[i];
    out[blockIdx.x * kMThreads + tid] = s;
    if (tid == 0) out[(1 << 20) + blockIdx.x] = (float)(t1 - t0) / (float)(iters - 1);
}

}  // namespace wrnn

using namespace wrnn;

template <int NS, int NC, int kDepth, int kEpi>
static void run_variant(const float *dW, float *dO, float *h) {
    const size_t lds = (kMWaves * kMStg + 3 * xcdm_pset(1)) * sizeof(float);
    hipFuncSetAttribute((const void *)variant_bench<NS, NC, kDepth, kEpi>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL((variant_bench<NS, NC, kDepth, kEpi>), dim3(256), dim3(kMThreads), lds, 0, dW, dO, 65);
    hipDeviceSynchronize();
    hipMemcpy(h, dO + (1 << 20), 256 * sizeof(float), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += h[i];
    m /= 256;
    printf("variant NS %d NC %d depth %d epilogue %d: %5.0f cycles (%5.1f per MFMA)\n", NS, NC, kDepth, kEpi, m, m / (NS * kMJ));
}

template <int NC, int kMode>
static void run_stream(const char *name, const float *dW, float *dO, float *h) {
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((stream_bench<NC, kMode>), dim3(256), dim3(kMThreads), 0, 0, dW, dO, 65);
    hipDeviceSynchronize();
    hipMemcpy(h, dO + (1 << 20), 256 * sizeof(float), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += h[i];
    m /= 256;
    printf("stream %-30s %5.0f cycles per 96 MFMAs: %5.1f each\n", name, m, m / 96);
}

template <int NQ, int S0, int NS>
static void run(const char *name, const float *dW, float *dO, float *h) {
    constexpr int kStgQ = xcdm_big(NQ) ? kMQuadMax : NQ;
    const size_t lds = (kMWaves * kStgQ * kMStg + 3 * xcdm_pset(NQ)) * sizeof(float);
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
    run_variant<3, 1, 2, 2>(dW, dO, h);
    run_variant<3, 1, 2, 1>(dW, dO, h);
    run_variant<3, 1, 2, 0>(dW, dO, h);
    run_variant<1, 2, 2, 2>(dW, dO, h);
    run_variant<1, 2, 4, 2>(dW, dO, h);
    run_variant<1, 4, 4, 2>(dW, dO, h);
    run_variant<3, 3, 2, 1>(dW, dO, h);
    run_variant<3, 3, 2, 0>(dW, dO, h);
    run_variant<3, 3, 3, 1>(dW, dO, h);
    run_variant<3, 3, 4, 1>(dW, dO, h);
    run_variant<3, 3, 8, 1>(dW, dO, h);
    run_variant<3, 3, 8, 0>(dW, dO, h);
    run_variant<3, 1, 4, 1>(dW, dO, h);
    run_variant<3, 1, 4, 0>(dW, dO, h);
    run_variant<1, 8, 2, 1>(dW, dO, h);
    run_variant<1, 8, 4, 1>(dW, dO, h);
    run_variant<1, 4, 4, 1>(dW, dO, h);
    run_variant<1, 2, 4, 1>(dW, dO, h);
    run_variant<1, 2, 4, 0>(dW, dO, h);
    run_stream<1, 0>("1 chain/set, one B", dW, dO, h);
    run_stream<1, 1>("1 chain/set, B[j]", dW, dO, h);
    run_stream<3, 0>("3 chains/set, one B", dW, dO, h);
    run_stream<3, 1>("3 chains/set, B[j]", dW, dO, h);
    run_stream<4, 1>("4 chains/set, B[j]", dW, dO, h);
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
