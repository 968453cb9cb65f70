// condition.hip — the producers and consumer on either side of the sample loop, on the device.
//
//  * upsample_pack_kernel: everything between MelResNet and the loop's time-major conditioning
//    records, in one pass over HBM (models/fatchord_version.py:82-89 UpsampleNetwork.forward
//    minus the MelResNet, the Stretch2d/Conv2d(1, 2s+1) chain of :71-79 incl. the zero padding
//    of pad_tensor :183-185, the crop by indent :88, resnet_stretch :83, fold_with_overlap
//    :293-340 and the cat/transpose the loop consumes, :190-205).  Output cond [win][B·nf][CD].
//  * postprocess_kernel: out [rows][steps] fp32 → the returned float64 waveform
//    (:243-258: decode_mu_law utils/dsp.py:98-103, xfade_and_unfold :342-405, trim, linear
//    fade-out), in float64 with the reference's operation order.
//
// Both are HBM-bound elementwise/stencil passes: one workgroup per tile of output steps, the
// upsampling cascade for the tile staged through LDS level by level, writes coalesced along
// the 208-float records.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "wavernn_amd.h"

namespace wrnn {

constexpr int kUpMaxScales = 4;
constexpr int kUpMaxScale = 15;
constexpr int kUpTile = 128;             // output steps per workgroup
constexpr int kUpThreads = 512;          // 8 waves; a wave writes one step's record at a time

struct UpArgs {
    const float *mel;     // [B][feat][T]   (unpadded; the pad frames are zeros)
    const float *aux;     // [B][A4][T]     MelResNet output (valid conv: T frames)
    float *cond;          // [win][B·nf][CD]
    int B, T, feat, A4, CD, pad, n_scales, hop, indent, L;
    int nf, stride, win, Lp;
    int scales[kUpMaxScales];
    int N[kUpMaxScales + 1];              // level lengths: N0 = T + 2·pad, Ni = N(i-1)·s_i
    int off[kUpMaxScales + 1];            // LDS offsets (floats) of levels 0 .. n-1, then the aux tile
    // Stretch(s) + Conv(1, 2s+1, pad s) as a 3-point stencil on the unstretched input:
    //   out[s·m + φ] = Σ_d pw[φ][d] · in[m − 1 + d],  pw[φ][d] = Σ_{j : ⌊(φ+j)/s⌋ = d} w[j]
    // (in[] = 0 outside [0, N), exactly the conv's zero padding of the stretched sequence)
    float pw[kUpMaxScales][3 * kUpMaxScale];
};

// VEC: feat and A4 multiples of 4 — a lane produces 4 consecutive columns, 16-B stores
template <bool VEC>
__global__ __launch_bounds__(kUpThreads) void upsample_pack_kernel(UpArgs a) {
    extern __shared__ float lvl[];
    const int t0 = blockIdx.x * kUpTile, t1 = min(t0 + kUpTile, a.Lp), b = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int kWaves = kUpThreads / 64;
    const int tv = min(t1, a.L);             // steps [t0, tv) carry signal, [tv, t1) fold padding
    const int n = a.n_scales, feat = a.feat, A4 = a.A4, CD = a.CD;
    int lo[kUpMaxScales + 1], hi[kUpMaxScales + 1];
    const int f0 = t0 / a.hop;               // first aux frame of the tile
    float *auxs = lvl + a.off[n];
    if (t0 < tv) {
        // rows each level provides for this tile (level n = the output, uncropped coordinates)
        lo[n] = t0 + a.indent;
        hi[n] = tv + a.indent;
        for (int i = n; i >= 1; --i) {
            const int s = a.scales[i - 1];
            lo[i - 1] = max(lo[i] / s - 1, 0);
            hi[i - 1] = min(a.N[i - 1], (hi[i] - 1) / s + 2);
        }
        // level 0: the zero-padded mel (pad_tensor, :183-185); the tile's aux frames
        for (int u = lo[0] + wave; u < hi[0]; u += kWaves) {
            const int tt = u - a.pad;
            for (int c = lane; c < feat; c += 64)
                lvl[a.off[0] + (u - lo[0]) * feat + c] =
                    (tt >= 0 && tt < a.T) ? a.mel[((size_t)b * feat + c) * a.T + tt] : 0.0f;
        }
        for (int f = f0 + wave; f <= (tv - 1) / a.hop; f += kWaves)
            for (int c = lane; c < A4; c += 64) auxs[(f - f0) * A4 + c] = a.aux[((size_t)b * A4 + c) * a.T + f];
        __syncthreads();
        // levels 1 .. n-1 (:71-79)
        for (int i = 1; i < n; ++i) {
            const int s = a.scales[i - 1], Np = a.N[i - 1], lp = lo[i - 1];
            const float *src = lvl + a.off[i - 1];
            float *dst = lvl + a.off[i];
            for (int q = lo[i] + wave; q < hi[i]; q += kWaves) {
                const int m = q / s, ph = q - m * s;
                const float w0 = a.pw[i - 1][3 * ph], w1 = a.pw[i - 1][3 * ph + 1], w2 = a.pw[i - 1][3 * ph + 2];
                const bool ok0 = m >= 1, ok2 = m + 1 < Np;
                for (int c = lane; c < feat; c += 64) {
                    const float x0 = ok0 ? src[(m - 1 - lp) * feat + c] : 0.0f;
                    const float x1 = src[(m - lp) * feat + c];
                    const float x2 = ok2 ? src[(m + 1 - lp) * feat + c] : 0.0f;
                    dst[(q - lo[i]) * feat + c] = fmaf(w2, x2, fmaf(w1, x1, w0 * x0));
                }
            }
            __syncthreads();
        }
    }
    // output level + aux stretch (:83) + fold scatter; one step's record per wave iteration
    const int s = a.scales[n - 1], Np = a.N[n - 1];
    const float *src = lvl + a.off[n - 1];
    const int Bo = a.B * a.nf;
    for (int p = t0 + wave; p < t1; p += kWaves) {
        const bool valid = p < a.L;
        int m = 0, lp = 0, fa = 0;
        float w0 = 0.0f, w1 = 0.0f, w2 = 0.0f;
        bool ok0 = false, ok2 = false;
        if (valid) {
            const int P = p + a.indent;
            m = P / s;
            const int ph = P - m * s;
            w0 = a.pw[n - 1][3 * ph];
            w1 = a.pw[n - 1][3 * ph + 1];
            w2 = a.pw[n - 1][3 * ph + 2];
            ok0 = m >= 1;
            ok2 = m + 1 < Np;
            lp = lo[n - 1];
            fa = p / a.hop - f0;
        }
        // every fold whose window [f·stride, f·stride + win) holds step p (at most two)
        const int fh = min(p / a.stride, a.nf - 1);
        if constexpr (VEC) {
            for (int c = 4 * lane; c < CD; c += 256) {
                float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (valid) {
                    if (c < feat) {
                        const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                        const float4 x0 = ok0 ? *reinterpret_cast<const float4 *>(src + (m - 1 - lp) * feat + c) : z;
                        const float4 x1 = *reinterpret_cast<const float4 *>(src + (m - lp) * feat + c);
                        const float4 x2 = ok2 ? *reinterpret_cast<const float4 *>(src + (m + 1 - lp) * feat + c) : z;
                        v.x = fmaf(w2, x2.x, fmaf(w1, x1.x, w0 * x0.x));
                        v.y = fmaf(w2, x2.y, fmaf(w1, x1.y, w0 * x0.y));
                        v.z = fmaf(w2, x2.z, fmaf(w1, x1.z, w0 * x0.z));
                        v.w = fmaf(w2, x2.w, fmaf(w1, x1.w, w0 * x0.w));
                    } else if (c < feat + A4) {
                        v = *reinterpret_cast<const float4 *>(auxs + fa * A4 + (c - feat));
                    }
                }
                for (int f = max(fh - 1, 0); f <= fh; ++f) {
                    const int tt = p - f * a.stride;
                    if (tt >= 0 && tt < a.win)
                        *reinterpret_cast<float4 *>(a.cond + ((size_t)tt * Bo + (size_t)b * a.nf + f) * CD + c) = v;
                }
            }
        } else {
            for (int c = lane; c < CD; c += 64) {
                float v = 0.0f;
                if (valid) {
                    if (c < feat) {
                        const float x0 = ok0 ? src[(m - 1 - lp) * feat + c] : 0.0f;
                        const float x1 = src[(m - lp) * feat + c];
                        const float x2 = ok2 ? src[(m + 1 - lp) * feat + c] : 0.0f;
                        v = fmaf(w2, x2, fmaf(w1, x1, w0 * x0));
                    } else if (c < feat + A4) {
                        v = auxs[fa * A4 + (c - feat)];
                    }
                }
                for (int f = max(fh - 1, 0); f <= fh; ++f) {
                    const int tt = p - f * a.stride;
                    if (tt >= 0 && tt < a.win) a.cond[((size_t)tt * Bo + (size_t)b * a.nf + f) * CD + c] = v;
                }
            }
        }
    }
}

struct PostArgs {
    const float *y;       // [rows][steps]
    double *wave;         // [wave_len]
    int rows, steps, batched, ov, stride, mu_law, wave_len, fade_len;
    double mu;            // n_classes − 1
    double fin_step, fout_step;  // linspace steps of the cross-fade and of the final fade
    int silence, xfade_len;
};

// numpy's linspace element: i·step + start, the last element exactly `stop`
__device__ inline double linspace_at(int i, int num, double start, double stop, double step) {
#pragma clang fp contract(off)
    if (num > 1 && i == num - 1) return stop;
    return (double)i * step + start;
}

__global__ void postprocess_kernel(PostArgs a) {
#pragma clang fp contract(off)
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.wave_len) return;
    auto mulaw = [&](double y) {
        // np.sign(y) / mu * ((1 + mu) ** np.abs(y) - 1)   (utils/dsp.py:102)
        const double sg = y > 0.0 ? 1.0 : (y < 0.0 ? -1.0 : 0.0);
        return sg / a.mu * (pow(a.mu + 1.0, fabs(y)) - 1.0);
    };
    double v;
    if (!a.batched) {
        v = (double)a.y[t];
        if (a.mu_law) v = mulaw(v);
    } else {
        // unfolded[start:end] += y[i] for i = 0, 1, ... (:399-403) after both fades (:396-397)
        v = 0.0;
        const int fh = min(t / a.stride, a.rows - 1);
        for (int f = max(fh - 1, 0); f <= fh; ++f) {
            const int k = t - f * a.stride;
            if (k < 0 || k >= a.steps) continue;
            double y = (double)a.y[(size_t)f * a.steps + k];
            if (a.mu_law) y = mulaw(y);
            if (k < a.ov) {
                const int q = k - a.silence;
                const double tt = q < 0 ? 0.0 : linspace_at(q, a.xfade_len, -1.0, 1.0, a.fin_step);
                y = y * (q < 0 ? 0.0 : sqrt(0.5 * (1.0 + tt)));
            }
            if (k >= a.steps - a.ov) {
                const int q = k - (a.steps - a.ov) - a.silence;
                const double tt = q < 0 ? 0.0 : linspace_at(q, a.xfade_len, -1.0, 1.0, a.fin_step);
                y = y * (q < 0 ? 1.0 : sqrt(0.5 * (1.0 - tt)));
            }
            v = v + y;
        }
    }
    // output[-20·hop:] *= np.linspace(1, 0, 20·hop)   (:255-258)
    const int q = t - (a.wave_len - a.fade_len);
    if (q >= 0) v = v * linspace_at(q, a.fade_len, 1.0, 0.0, a.fout_step);
    a.wave[t] = v;
}

// error of the last failed stateless call on this thread (also capi.cpp's wrnn_philox_draws)
thread_local std::string g_cond_err;
int cond_fail(int code, const std::string &m) {
    g_cond_err = m;
    return code;
}

namespace {

// fold geometry of fold_with_overlap (:317-330): folds, stride, window, padded length
void fold_geometry(int L, int target, int overlap, int *nf, int *stride, int *win, int *Lp) {
    if (target <= 0) {
        *nf = 1;
        *stride = L;
        *win = L;
        *Lp = L;
        return;
    }
    int n = (L - overlap) / (target + overlap);
    const int ext = n * (target + overlap) + overlap;
    if (L - ext != 0) ++n;
    *nf = n;
    *stride = target + overlap;
    *win = target + 2 * overlap;
    *Lp = (n - 1) * (target + overlap) + target + 2 * overlap;
}

int check_up(const wrnn_upsample_cfg *c) {
    if (!c) return cond_fail(WRNN_EINVAL, "null upsample config");
    if (c->n_scales < 1 || c->n_scales > kUpMaxScales) return cond_fail(WRNN_EINVAL, "n_scales must be 1..4");
    for (int i = 0; i < c->n_scales; ++i) {
        if (c->scales[i] < 1 || c->scales[i] > kUpMaxScale)
            return cond_fail(WRNN_EUNSUPPORTED, "upsample scale must be 1..15");
        if (!c->taps[i]) return cond_fail(WRNN_EINVAL, "missing upsample taps (upsample.up_layers.*.weight)");
    }
    if (c->feat_dims < 1 || c->res_out_dims < 0 || c->pad < 0) return cond_fail(WRNN_EINVAL, "bad dims");
    return WRNN_OK;
}
}  // namespace

}  // namespace wrnn

extern "C" {

const char *wrnn_cond_last_error(void) { return wrnn::g_cond_err.c_str(); }

int wrnn_cond_shape(const wrnn_upsample_cfg *cfg, int B, int T, int target, int overlap, int *steps, int *rows) {
    using namespace wrnn;
    if (int rc = check_up(cfg)) return rc;
    if (B < 1 || T < 1) return cond_fail(WRNN_EINVAL, "B and T must be >= 1");
    int hop = 1;
    for (int i = 0; i < cfg->n_scales; ++i) hop *= cfg->scales[i];
    const long long L = (long long)hop * T;
    if (L > (1LL << 30)) return cond_fail(WRNN_EINVAL, "utterance too long");
    if (target > 0 && (overlap < 0 || L < overlap)) return cond_fail(WRNN_EINVAL, "bad target/overlap");
    int nf, stride, win, Lp;
    fold_geometry((int)L, target, overlap, &nf, &stride, &win, &Lp);
    if (steps) *steps = win;
    if (rows) *rows = B * nf;
    return WRNN_OK;
}

int wrnn_upsample_pack(const wrnn_upsample_cfg *cfg, const float *mel, const float *aux, int B, int T, int target,
                       int overlap, float *cond, void *stream) {
    using namespace wrnn;
    int win = 0, rows = 0;
    if (int rc = wrnn_cond_shape(cfg, B, T, target, overlap, &win, &rows)) return rc;
    if (!mel || !cond || (cfg->res_out_dims > 0 && !aux)) return cond_fail(WRNN_EINVAL, "null tensor");
    UpArgs a{};
    a.mel = mel;
    a.aux = aux;
    a.cond = cond;
    a.B = B;
    a.T = T;
    a.feat = cfg->feat_dims;
    a.A4 = cfg->res_out_dims;
    a.CD = a.feat + a.A4;
    a.pad = cfg->pad;
    a.n_scales = cfg->n_scales;
    a.hop = 1;
    a.N[0] = T + 2 * cfg->pad;
    for (int i = 0; i < a.n_scales; ++i) {
        const int s = cfg->scales[i];
        a.scales[i] = s;
        a.hop *= s;
        a.N[i + 1] = a.N[i] * s;
        // taps (host) → per-phase 3-point stencil weights, summed in double
        for (int ph = 0; ph < s; ++ph) {
            double acc[3] = {0.0, 0.0, 0.0};
            for (int j = 0; j < 2 * s + 1; ++j) acc[(ph + j) / s] += (double)cfg->taps[i][j];
            for (int d = 0; d < 3; ++d) a.pw[i][3 * ph + d] = (float)acc[d];
        }
    }
    a.indent = cfg->pad * a.hop;
    a.L = a.hop * T;
    fold_geometry(a.L, target, overlap, &a.nf, &a.stride, &a.win, &a.Lp);
    // LDS rows per level: m rows of level i need <= m / s_i + 4 rows of level i-1
    int cap[kUpMaxScales], m = kUpTile, off = 0;
    for (int i = a.n_scales; i >= 1; --i) {
        m = m / a.scales[i - 1] + 5;
        cap[i - 1] = m;
    }
    for (int i = 0; i < a.n_scales; ++i) {
        a.off[i] = off;
        off += cap[i] * a.feat;
    }
    a.off[a.n_scales] = off;                       // aux frames of the tile
    off += (kUpTile / a.hop + 2) * a.A4;
    const size_t lds = (size_t)off * 4;
    if (lds > 160 * 1024) return cond_fail(WRNN_EUNSUPPORTED, "upsample tile exceeds LDS");
    const bool vec = a.feat % 4 == 0 && a.A4 % 4 == 0;
    const void *kern = vec ? (const void *)upsample_pack_kernel<true> : (const void *)upsample_pack_kernel<false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return cond_fail(WRNN_EHIP, hipGetErrorString(e));
    }
    const dim3 grid((a.Lp + kUpTile - 1) / kUpTile, B);
    if (vec) hipLaunchKernelGGL(upsample_pack_kernel<true>, grid, dim3(kUpThreads), lds, (hipStream_t)stream, a);
    else hipLaunchKernelGGL(upsample_pack_kernel<false>, grid, dim3(kUpThreads), lds, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? WRNN_OK : cond_fail(WRNN_EHIP, hipGetErrorString(e));
}

int wrnn_postprocess(const float *y, int rows, int steps, int batched, int overlap, int mu_law, int n_classes,
                     int wave_len, int fade_len, double *wave, void *stream) {
    using namespace wrnn;
    if (!y || !wave || rows < 1 || steps < 1 || wave_len < 1) return cond_fail(WRNN_EINVAL, "bad arguments");
    if (fade_len < 1 || fade_len > wave_len)
        return cond_fail(WRNN_EINVAL, "operands could not be broadcast together: the fade-out (20*hop_length = " +
                                          std::to_string(fade_len) + ") is longer than the waveform (" +
                                          std::to_string(wave_len) + ")");
    PostArgs a{};
    a.y = y;
    a.wave = wave;
    a.rows = rows;
    a.steps = steps;
    a.batched = batched != 0;
    a.mu_law = mu_law != 0;
    a.mu = (double)(n_classes - 1);
    a.wave_len = wave_len;
    a.fade_len = fade_len;
    a.fout_step = (0.0 - 1.0) / (double)(fade_len > 1 ? fade_len - 1 : 1);
    if (a.batched) {
        const int target = steps - 2 * overlap;
        if (overlap < 0 || target < 1) return cond_fail(WRNN_EINVAL, "bad overlap for the fold length");
        const long long total = (long long)rows * (target + overlap) + overlap;
        if (wave_len > total) return cond_fail(WRNN_EINVAL, "wave_len exceeds the unfolded length");
        a.ov = overlap;
        a.stride = target + overlap;
        a.silence = overlap / 2;
        a.xfade_len = overlap - a.silence;
        a.fin_step = 2.0 / (double)(a.xfade_len > 1 ? a.xfade_len - 1 : 1);
    } else if (wave_len > steps) {
        return cond_fail(WRNN_EINVAL, "wave_len exceeds the generated length");
    }
    hipLaunchKernelGGL(postprocess_kernel, dim3((wave_len + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? WRNN_OK : cond_fail(WRNN_EHIP, hipGetErrorString(e));
}

}  // extern "C"
