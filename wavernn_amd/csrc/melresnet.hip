// melresnet.hip — the UpsampleNetwork's MelResNet (models/fatchord_version.py:13-48) in inference
// form as ONE kernel: conv_in (k = 2·pad + 1, no padding) → BatchNorm → ReLU → res_blocks ×
// [1×1 conv → BN → ReLU → 1×1 conv → BN → + residual] → conv_out (1×1, bias), every BatchNorm
// (eval: running statistics) folded into the preceding conv's weights and a bias on the host
// (condition.py: melresnet_pack).  The torch module is 2 + 2·res_blocks convolutions and as many
// BatchNorm / ReLU / add kernels (≈ 80 launches at res_blocks = 10); here a workgroup carries a tile
// of kMrF frames of one utterance through all layers with the activations in LDS.
//
// Packed weights (floats), every matrix k-major ("Wt[k][out]": a wave's 64 lanes read 64
// consecutive outputs of one k, coalesced):
//   conv_in  Wt[(c·K + tap)][C], bias[C]          (K = 2·pad + 1, c < in_dims)
//   block i  Wt1[C][C], b1[C], Wt2[C][C], b2[C]
//   conv_out Wt[C][R], bias[R]
// Layer outputs: thread t owns output row t % Cout and Cout·kMrF / 256 consecutive frames; each
// layer's weights pass through LDS 128 input channels at a time (every thread loading its share at
// once: one round trip per chunk), read back conflict-free (a wave's lanes: consecutive outputs)
// while the activations are LDS broadcasts (a wave's lanes share the frames).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "wavernn_amd.h"

namespace wrnn {

constexpr int kMrThreads = 256;
// frames per workgroup: 16 when the grid has enough tiles to fill the chip, else 4 (a single 5 s mel
// is 26 tiles of 16 frames on 256 CUs; at 4 frames it is 102, each carrying a quarter of the work)
constexpr int kMrFBig = 16, kMrFSmall = 4;

constexpr int kMrKc = 128;        // weight rows (input channels) staged through LDS at a time

// Rows [k0, k0 + kc) of a k-major weight matrix (Cout wide) → LDS, every thread loading its share
// at once (one round trip per chunk instead of one per input channel)
__device__ __forceinline__ void mr_stage(const float *__restrict__ Wt, int k0, int kc, int Cout, float *wbuf) {
    __syncthreads();
    const float *src = Wt + (size_t)k0 * Cout;
    const int n = kc * Cout;
    if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        for (int i = 4 * threadIdx.x; i < n; i += 4 * kMrThreads)
            *reinterpret_cast<float4 *>(wbuf + i) = *reinterpret_cast<const float4 *>(src + i);
    } else {
        for (int i = threadIdx.x; i < n; i += kMrThreads) wbuf[i] = src[i];
    }
    __syncthreads();
}

// acc = bias + W·in over the thread's frames, the weights staged through LDS chunk by chunk.
// `live`: this thread owns outputs (all threads stage).  X(k, i): input k at the thread's frame i.
template <int FPT, typename X>
__device__ __forceinline__ void mr_layer(const float *__restrict__ Wt, const float *__restrict__ bias, int Kin,
                                         int Cout, float *wbuf, bool live, int row, float (&acc)[FPT], X x) {
    if (live) {
#pragma unroll
        for (int i = 0; i < FPT; ++i) acc[i] = bias[row];
    }
    for (int k0 = 0; k0 < Kin; k0 += kMrKc) {
        const int kc = min(kMrKc, Kin - k0);
        mr_stage(Wt, k0, kc, Cout, wbuf);
        if (live) {
            for (int k = 0; k < kc; ++k) {
                const float w = wbuf[k * Cout + row];
#pragma unroll
                for (int i = 0; i < FPT; ++i) acc[i] = fmaf(w, x(k0 + k, i), acc[i]);
            }
        }
    }
}

struct MrArgs {
    const float *w;       // packed weights (device)
    const float *mel;     // [U][in_dims][T + 2·pad]  the pad_tensor'd mel
    float *aux;           // [U][R][T]
    int U, T, in_dims, C, R, blocks, K;
};

template <int kMrF, int FPT_C, int FPT_R>
__global__ __launch_bounds__(kMrThreads) void melresnet_kernel(MrArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int u = blockIdx.y, t0 = blockIdx.x * kMrF, tid = threadIdx.x;
    const int Tp = a.T + a.K - 1, KF = kMrF + a.K - 1;
    float *act = lds;                              // [C][kMrF]
    float *tmp = act + a.C * kMrF;                 // [C][kMrF]
    float *wbuf = tmp + a.C * kMrF;                // [kMrKc][max(C, R)]
    float *xin = wbuf + kMrKc * max(a.C, a.R);     // [in_dims][kMrF + K − 1]  the mel tile (+ halo)
    for (int i = tid; i < a.in_dims * KF; i += kMrThreads) {
        const int c = i / KF, f = i - c * KF;
        xin[i] = t0 + f < Tp ? a.mel[((size_t)u * a.in_dims + c) * Tp + t0 + f] : 0.0f;
    }
    const int row = tid % a.C, fc = (tid / a.C) * FPT_C;
    const bool live_c = tid < a.C * (kMrF / FPT_C);
    const float *W = a.w;
    float acc[FPT_C];
    // conv_in + BN + ReLU: input k = c·K + tap reads frame f + tap of the tile
    const int Kin0 = a.in_dims * a.K;
    mr_layer<FPT_C>(W, W + (size_t)Kin0 * a.C, Kin0, a.C, wbuf, live_c, row, acc, [&](int k, int i) {
        const int c = k / a.K;
        return xin[c * KF + (k - c * a.K) + fc + i];
    });
    if (live_c) {
#pragma unroll
        for (int i = 0; i < FPT_C; ++i) act[row * kMrF + fc + i] = fmaxf(acc[i], 0.0f);
    }
    W += (size_t)Kin0 * a.C + a.C;
    for (int blk = 0; blk < a.blocks; ++blk) {
        // (mr_stage's leading barrier orders these layers' LDS reads after the previous writes)
        mr_layer<FPT_C>(W, W + (size_t)a.C * a.C, a.C, a.C, wbuf, live_c, row, acc,
                        [&](int k, int i) { return act[k * kMrF + fc + i]; });
        if (live_c) {
#pragma unroll
            for (int i = 0; i < FPT_C; ++i) tmp[row * kMrF + fc + i] = fmaxf(acc[i], 0.0f);
        }
        W += (size_t)a.C * a.C + a.C;
        mr_layer<FPT_C>(W, W + (size_t)a.C * a.C, a.C, a.C, wbuf, live_c, row, acc,
                        [&](int k, int i) { return tmp[k * kMrF + fc + i]; });
        __syncthreads();   // every thread has read act (conv1 above) before it is overwritten
        if (live_c) {
#pragma unroll
            for (int i = 0; i < FPT_C; ++i) act[row * kMrF + fc + i] = acc[i] + act[row * kMrF + fc + i];
        }
        W += (size_t)a.C * a.C + a.C;
    }
    // conv_out (bias) → aux
    const int orow = tid % a.R, fr = (tid / a.R) * FPT_R;
    const bool live_r = tid < a.R * (kMrF / FPT_R);
    float acc_r[FPT_R];
    mr_layer<FPT_R>(W, W + (size_t)a.C * a.R, a.C, a.R, wbuf, live_r, orow, acc_r,
                    [&](int k, int i) { return act[k * kMrF + fr + i]; });
    if (live_r) {
#pragma unroll
        for (int i = 0; i < FPT_R; ++i)
            if (t0 + fr + i < a.T) a.aux[((size_t)u * a.R + orow) * a.T + t0 + fr + i] = acc_r[i];
    }
}

// frames per thread for Cout outputs over kMrF frames and 256 threads (0: unsupported)
inline int mr_fpt(int cout, int kMrF) {
    if (cout < 1 || cout > kMrThreads) return 0;
    const int out = cout * kMrF;
    if (out <= kMrThreads) return 1;
    if (out % kMrThreads) return 0;
    const int f = out / kMrThreads;
    return kMrF % f == 0 ? f : 0;
}

}  // namespace wrnn

extern "C" {

int wrnn_melresnet_floats(const wrnn_melresnet_cfg *cfg) {
    if (!cfg || cfg->in_dims < 1 || cfg->compute_dims < 1 || cfg->res_out_dims < 1 || cfg->res_blocks < 0 ||
        cfg->pad < 0)
        return -1;
    const long long C = cfg->compute_dims, R = cfg->res_out_dims, K = 2LL * cfg->pad + 1;
    return (int)(cfg->in_dims * K * C + C + cfg->res_blocks * 2 * (C * C + C) + C * R + R);
}

namespace {
// CUs of the current device, queried once per device (a partitioned part reports fewer)
int mr_num_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        cus[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
    }
    return cus[dev];
}

// The tile form for U utterances of T frames: 16-frame tiles, or 4-frame tiles when the 16-frame
// grid has fewer workgroups than the device has CUs (WRNN_MR_FRAMES=16|4 forces one).  Sets the
// frames-per-thread of the compute / output layers; false when the channel counts fit neither.
bool mr_choose(const wrnn_melresnet_cfg *cfg, int U, int T, int *F_, int *fc_, int *fr_, size_t *lds_) {
    using namespace wrnn;
    const int K = 2 * cfg->pad + 1;
    const char *fe = std::getenv("WRNN_MR_FRAMES");
    int F = (long long)U * ((T + kMrFBig - 1) / kMrFBig) >= mr_num_cus() ? kMrFBig : kMrFSmall;
    if (fe && (std::atoi(fe) == kMrFBig || std::atoi(fe) == kMrFSmall)) F = std::atoi(fe);
    int fc = mr_fpt(cfg->compute_dims, F), fr = mr_fpt(cfg->res_out_dims, F);
    if ((!fc || !fr) && F == kMrFSmall) {   // channel counts only the 16-frame form covers
        F = kMrFBig;
        fc = mr_fpt(cfg->compute_dims, F);
        fr = mr_fpt(cfg->res_out_dims, F);
    }
    const size_t lds = ((size_t)cfg->in_dims * (F + K - 1) + 2 * (size_t)cfg->compute_dims * F +
                        (size_t)kMrKc * std::max(cfg->compute_dims, cfg->res_out_dims)) * 4;
    *F_ = F, *fc_ = fc, *fr_ = fr, *lds_ = lds;
    return fc && fr && lds <= 160 * 1024;
}
}  // namespace

int wrnn_melresnet_tile_frames(const wrnn_melresnet_cfg *cfg, int U, int T) {
    if (wrnn_melresnet_floats(cfg) < 0 || U < 1 || T < 1) return WRNN_EINVAL;
    int F = 0, fc = 0, fr = 0;
    size_t lds = 0;
    return mr_choose(cfg, U, T, &F, &fc, &fr, &lds) ? F : WRNN_EUNSUPPORTED;
}

int wrnn_melresnet(const wrnn_melresnet_cfg *cfg, const float *packed, const float *mel, int U, int T, float *aux,
                   void *stream) {
    using namespace wrnn;
    if (wrnn_melresnet_floats(cfg) < 0 || !packed || !mel || !aux || U < 1 || T < 1) return WRNN_EINVAL;
    const int K = 2 * cfg->pad + 1;
    int F = 0, fc = 0, fr = 0;
    size_t lds = 0;
    if (!mr_choose(cfg, U, T, &F, &fc, &fr, &lds)) return WRNN_EUNSUPPORTED;
    MrArgs a{packed, mel, aux, U, T, cfg->in_dims, cfg->compute_dims, cfg->res_out_dims, cfg->res_blocks, K};
    const dim3 grid((T + F - 1) / F, U);
    hipStream_t st = (hipStream_t)stream;
#define WRNN_MR_CASE(FF, A, B)                                                                      \
    if (F == FF && fc == A && fr == B) {                                                            \
        if (lds > 64 * 1024 &&                                                                      \
            hipFuncSetAttribute((const void *)melresnet_kernel<FF, A, B>,                           \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) \
            return WRNN_EHIP;                                                                       \
        hipLaunchKernelGGL((melresnet_kernel<FF, A, B>), grid, dim3(kMrThreads), lds, st, a);       \
        return hipGetLastError() == hipSuccess ? WRNN_OK : WRNN_EHIP;                              \
    }
    WRNN_MR_CASE(16, 8, 8) WRNN_MR_CASE(16, 1, 1) WRNN_MR_CASE(16, 2, 2) WRNN_MR_CASE(16, 4, 4)
    WRNN_MR_CASE(16, 16, 16) WRNN_MR_CASE(16, 8, 1) WRNN_MR_CASE(16, 8, 2) WRNN_MR_CASE(16, 8, 4)
    WRNN_MR_CASE(16, 8, 16) WRNN_MR_CASE(16, 1, 8) WRNN_MR_CASE(16, 2, 8) WRNN_MR_CASE(16, 4, 8)
    WRNN_MR_CASE(16, 16, 8)
    WRNN_MR_CASE(4, 2, 2) WRNN_MR_CASE(4, 1, 1) WRNN_MR_CASE(4, 4, 4) WRNN_MR_CASE(4, 2, 1)
    WRNN_MR_CASE(4, 1, 2) WRNN_MR_CASE(4, 4, 2) WRNN_MR_CASE(4, 2, 4) WRNN_MR_CASE(4, 4, 1)
    WRNN_MR_CASE(4, 1, 4)
#undef WRNN_MR_CASE
    return WRNN_EUNSUPPORTED;
}

}  // extern "C"
