// fatchord_loop.hip — persistent CDNA4 kernel for the WaveRNN sample loop.
//
// Replaces the host-driven loop of models/fatchord_version.py:201-241 (≈40 eager torch
// launches per sample) by ONE launch that runs all L steps on chip:
//
//   * grid = G workgroups (one per CU), all co-resident; workgroup w owns hidden units
//     [w·U, w·U+U) of both GRUs (their r/z/n gate rows of W_ih and W_hh), fc1/fc2 rows
//     [w·UF, …) and (RAW) fc3 rows [w·UC, …).  Its weight slab lives in LDS for the whole
//     launch, so HBM carries only the per-step conditioning (≈2.4 KB/row-step).
//   * the four all-to-all dependencies of a step (h1 → GRU2, h2 → fc1, f1 → fc2, f2 →
//     fc3; plus logits → sampler in RAW) are hand-offs through 8-byte {tag, value}
//     granules: one agent-scope (sc1) store per value, polled by sc1 loads until the tag
//     equals the step (MI355X_MICROARCH.md, R2 hand-off: no fence, placement-independent).
//   * MoL's fc3 (30 rows) and every sampler are computed redundantly and bit-identically in
//     every workgroup, so the sampled x_{t} never needs a hand-off of its own.
//   * every wait is bounded (s_memrealtime); a timeout sets an abort word that every other
//     workgroup sees, so a non-resident grid or fault ends the kernel instead of hanging it.
//
// Arithmetic is fp32 throughout (bf16 weights flip RAW labels).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fatchord_loop.h"

namespace wrnn {

// ------------------------------------------------------------------ wave-level helpers
#define WRNN_DPP(v, ctrl) \
    __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, (v)), (ctrl), 0xF, 0xF, false))

// Full-wave sum; every lane returns the same bits.  Row stages via DPP (xor1, xor2,
// half-mirror, mirror), then the four row sums combined in a fixed order.
__device__ __forceinline__ float wave_sum(float v) {
    v += WRNN_DPP(v, 0xB1);    // quad_perm [1,0,3,2]
    v += WRNN_DPP(v, 0x4E);    // quad_perm [2,3,0,1]
    v += WRNN_DPP(v, 0x141);   // row_half_mirror
    v += WRNN_DPP(v, 0x140);   // row_mirror
    float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
    float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
    float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
    return (r0 + r1) + (r2 + r3);
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, WRNN_DPP(v, 0xB1));
    v = fmaxf(v, WRNN_DPP(v, 0x4E));
    v = fmaxf(v, WRNN_DPP(v, 0x141));
    v = fmaxf(v, WRNN_DPP(v, 0x140));
    float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
    float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
    float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// (value, index) argmax: larger value wins, ties go to the smaller index (torch: first max).
__device__ __forceinline__ void am_merge(float &v, int &i, float ov, int oi) {
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}

__device__ __forceinline__ int wave_argmax(float v, int i) {
#define WRNN_AM_STAGE(ctrl)                                                           \
    {                                                                                 \
        float ov = WRNN_DPP(v, ctrl);                                                 \
        int oi = __builtin_amdgcn_mov_dpp(i, (ctrl), 0xF, 0xF, false);                \
        am_merge(v, i, ov, oi);                                                       \
    }
    WRNN_AM_STAGE(0xB1) WRNN_AM_STAGE(0x4E) WRNN_AM_STAGE(0x141) WRNN_AM_STAGE(0x140)
#undef WRNN_AM_STAGE
    float bv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        float ov = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), r));
        int oi = __builtin_amdgcn_readlane(i, r);
        am_merge(bv, bi, ov, oi);
    }
    return bi;
}

// NR dot products against one shared vector: acc[r] += W[r]·x over K4 float4 chunks,
// row r at w0 + r·wstride.  Lane l takes chunks l, l+64, … (contiguous 16 B per lane:
// conflict-free ds_read_b128).
template <int NR>
__device__ __forceinline__ void dots(const float *__restrict__ w0, int wstride, const float *__restrict__ x,
                                     int K4, int lane, float (&acc)[NR]) {
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    for (int c = lane; c < K4; c += 64) {
        const float4 xv = x4[c];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const float4 wv = reinterpret_cast<const float4 *>(w0 + r * wstride)[c];
            float a = acc[r];
            a = fmaf(wv.x, xv.x, a);
            a = fmaf(wv.y, xv.y, a);
            a = fmaf(wv.z, xv.z, a);
            a = fmaf(wv.w, xv.w, a);
            acc[r] = a;
        }
    }
}

__device__ __forceinline__ float sigmoid_(float x) { return 1.0f / (1.0f + expf(-x)); }

// ------------------------------------------------------------------------------ Philox
__device__ __forceinline__ uint32_t philox_word(unsigned long long seed, unsigned long long row,
                                                uint32_t step, uint32_t k) {
    uint32_t c0 = k >> 2, c1 = step, c2 = (uint32_t)row, c3 = (uint32_t)(row >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    const uint32_t w = k & 3;
    return w == 0 ? c0 : w == 1 ? c1 : w == 2 ? c2 : c3;
}

// Draw k of row/step in the reference distribution (MOL: U(1e-5, 1-1e-5); RAW: Exp(1)).
__device__ __forceinline__ float philox_noise(unsigned long long seed, unsigned long long row,
                                              uint32_t step, uint32_t k, int mol) {
    const uint32_t w = philox_word(seed, row, step, k);
    if (mol) return 1e-5f + (1.0f - 2e-5f) * ((float)(w >> 8) * 0x1p-24f);
    return -logf((float)((w >> 8) + 1u) * 0x1p-24f);
}

// ---------------------------------------------------------------------------- hand-off
__device__ __forceinline__ void publish(unsigned long long *g, uint32_t tag, float v) {
    const unsigned long long x = ((unsigned long long)tag << 32) | __float_as_uint(v);
    __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __noinline__ void record_abort(int *ctl, int code, int step, int hop, int wg) {
    if (atomicCAS(&ctl[1], 0, code) == 0) {
        ctl[2] = step;
        ctl[3] = hop;
        ctl[4] = wg;
    }
    __hip_atomic_store(&ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Gather n = Bc·N granules of one hop into LDS rows (row b at dst + b·ld); called by the
// kPollThreads polling threads only.  Each thread keeps all its outstanding polls in flight
// per pass.  On timeout, or when another workgroup has aborted, sets *lds_abort.
__device__ void gather(const unsigned long long *g, int n, int N, float *dst, int ld, uint32_t tag,
                       int *ctl, long long timeout, int step, int hop, int *lds_abort) {
    const int tid = threadIdx.x;
    const int mine = (n - tid + kPollThreads - 1) / kPollThreads;  // tid < kPollThreads
    unsigned long long v[kGatherMax];
    const uint32_t all = (mine <= 0) ? 0u : (mine >= 32 ? 0xFFFFFFFFu : ((1u << mine) - 1u));
    uint32_t done = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    while (done != all) {
#pragma unroll
        for (int k = 0; k < kGatherMax; ++k)
            if (k < mine && !(done & (1u << k)))
                v[k] = __hip_atomic_load(g + tid + k * kPollThreads, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < kGatherMax; ++k)
            if (k < mine && !(done & (1u << k)) && (uint32_t)(v[k] >> 32) == tag) {
                const int i = tid + k * kPollThreads;
                const int b = i / N, j = i - b * N;
                dst[b * ld + j] = __uint_as_float((uint32_t)v[k]);
                done |= 1u << k;
            }
        if (done == all) break;
        if ((++spins & 31u) == 0) {
            const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout;
            const bool other = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (late || other) {
                if (late) record_abort(ctl, -4, step, hop, blockIdx.x);
                *lds_abort = 1;
                break;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Stage work item `it` → wave: items 0,1 go to the publishing waves 2,3 first.
__device__ __forceinline__ int first_item(int wave) { return (wave + 2) & (kWaves - 1); }

// One GRU cell (ATen gru_cell order, verified bit-exact vs torch.nn.GRUCell on CPU):
// r = σ(hr + ir), z = σ(hz + iz), n = tanh(in + hn·r), h' = (h − n)·z + n.
__device__ __forceinline__ float gru_unit(const float *S, int o_wih, int o_whh, int o_bih, int o_bhh, int U,
                                          int u, const float *x, int KI, const float *h, int R, float h_old,
                                          int lane) {
    float ai[3] = {0.f, 0.f, 0.f}, ah[3] = {0.f, 0.f, 0.f};
    dots<3>(S + o_wih + u * KI, U * KI, x, KI / 4, lane, ai);
    dots<3>(S + o_whh + u * R, U * R, h, R / 4, lane, ah);
    float gi[3], gh[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        gi[g] = wave_sum(ai[g]) + S[o_bih + g * U + u];
        gh[g] = wave_sum(ah[g]) + S[o_bhh + g * U + u];
    }
    const float r = sigmoid_(gh[0] + gi[0]);
    const float z = sigmoid_(gh[1] + gi[1]);
    const float n = tanhf(gi[2] + gh[2] * r);
    return (h_old - n) * z + n;
}

// LDS-only workgroup barrier.  Unlike __syncthreads() it does not drain vmcnt, so the loader
// wave's LDS-DMA and the publishers' granule stores stay in flight across it.
__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

#define WRNN_GPTR(p) ((__attribute__((address_space(1))) void *)(p))
#define WRNN_LPTR(p) ((__attribute__((address_space(3))) void *)(p))

// ------------------------------------------------------------------------ the loop kernel
__global__ __launch_bounds__(kThreads) void fatchord_loop_kernel(LoopArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int w = blockIdx.x;
    const int R = a.R, F = a.F, A = a.A, Bc = a.Bc, NK = a.NK;
    const LdsLayout ll = lds_layout(a.s.total, Bc, R, F, A, a.NC, NK);
    float *S = smem + ll.slab;
    float *h1 = smem + ll.h1, *h2 = smem + ll.h2, *xa = smem + ll.xa, *fa = smem + ll.fa;
    float *f2 = smem + ll.f2, *lg = smem + ll.lg, *pre = smem + ll.pre, *xprev = smem + ll.xprev;
    int *lbl = reinterpret_cast<int *>(smem + ll.lbl);
    int *abort_flag = reinterpret_cast<int *>(smem + ll.flag);
    const int RA = R + A, FA = F + A, PP = ll.pp, P = R + 3 * A + NK;
    const int Uv = min(a.U, R - w * a.U);                 // valid units here
    const int UFv = max(0, min(a.UF, F - w * a.UF));
    const int UCv = a.mol ? 0 : max(0, min(a.UC, a.NC - w * a.UC));
    const bool loader = wave == kLoaderWave;
    const bool compute = !loader;
    const bool poller = tid < kPollThreads;

    // ---- prologue: weights → LDS, zero state, step-0 record [cI (R) | a2 a3 a4 (3A) | noise (NK)]
    {
        const float4 *src = reinterpret_cast<const float4 *>(a.slab + (size_t)w * a.s.total);
        float4 *dst = reinterpret_cast<float4 *>(S);
        for (int i = tid; i < a.s.total / 4; i += kThreads) dst[i] = src[i];
        for (int i = tid; i < Bc * R; i += kThreads) { h1[i] = 0.0f; h2[i] = 0.0f; }
        if (tid < Bc) { xprev[tid] = 0.0f; lbl[tid] = 0; }   // x = zeros (fatchord_version.py:196)
        if (tid == 0) *abort_flag = 0;
        for (int i = tid; i < Bc * P; i += kThreads) {
            const int b = i / P, q = i - b * P;
            const size_t row = (size_t)a.b0 + b;              // t = 0
            float v;
            if (q < R) v = a.cI[(size_t)b * R + q];
            else if (q < R + 3 * A) v = a.cond[row * a.CD + a.feat + A + (q - R)];
            else if (a.noise) v = a.noise[row * NK + (q - R - 3 * A)];
            else v = philox_noise(a.seed, (unsigned long long)(a.row0 + b), 0u, (uint32_t)(q - R - 3 * A), a.mol);
            pre[b * PP + q] = v;
        }
    }
    __syncthreads();

    const float *wi0 = S + a.s.wi0;
    const size_t hop_stride = (size_t)Bc * a.NMAX;
    unsigned long long *xgH1 = a.xg + HOP_H1 * hop_stride, *xgH2 = a.xg + HOP_H2 * hop_stride;
    unsigned long long *xgF1 = a.xg + HOP_F1 * hop_stride, *xgF2 = a.xg + HOP_F2 * hop_stride;
    unsigned long long *xgLG = a.xg + HOP_LOGITS * hop_stride;
    const int it0 = first_item(wave);
    const bool writer = loader && w == 0 && lane < Bc;

    for (int t = 0; t < a.L; ++t) {
        const uint32_t tag = (uint32_t)t + 1u;
        const float *cur = pre + (t & 1) * Bc * PP;
        float *nxt = pre + ((t + 1) & 1) * Bc * PP;
        const bool has_next = (t + 1) < a.L;

        if (loader) {
            // outputs of step t-1 (LDS reads happen before any DMA is in flight)
            if (writer && t > 0) {
                const size_t o = (size_t)(a.b0 + lane) * a.L + (t - 1);
                a.out[o] = xprev[lane];
                if (a.labels) a.labels[o] = lbl[lane];
            }
            if (has_next) {
                const int t1 = t + 1;
                for (int b = 0; b < Bc; ++b) {
                    float *dst = nxt + b * PP;
                    const size_t row = (size_t)t1 * a.Bt + a.b0 + b;
                    if (!a.noise)   // Philox draws: plain LDS writes, issued before the DMAs
                        for (int k = lane; k < NK; k += 64)
                            dst[R + 3 * A + k] = philox_noise(a.seed, (unsigned long long)(a.row0 + b),
                                                              (uint32_t)t1, (uint32_t)k, a.mol);
                    const float *ci = a.cI + ((size_t)t1 * Bc + b) * R;
                    for (int c = 0; c < R; c += 256)
                        if (c + lane * 4 < R)
                            __builtin_amdgcn_global_load_lds(WRNN_GPTR(ci + c + lane * 4), WRNN_LPTR(dst + c), 16, 0, 0);
                    const float *ax = a.cond + row * a.CD + a.feat + A;
                    for (int c = 0; c < 3 * A; c += 64)
                        if (c + lane < 3 * A)
                            __builtin_amdgcn_global_load_lds(WRNN_GPTR(ax + c + lane), WRNN_LPTR(dst + R + c), 4, 0, 0);
                    if (a.noise) {
                        const float *nz = a.noise + row * NK;
                        for (int c = 0; c < NK; c += 64)
                            if (c + lane < NK)
                                __builtin_amdgcn_global_load_lds(WRNN_GPTR(nz + c + lane),
                                                                 WRNN_LPTR(dst + R + 3 * A + c), 4, 0, 0);
                    }
                }
            }
        }

        // S1: x = I([x_{t-1}; m_t; a1_t]) = cI_t + W_I[:,0]·x_{t-1}; stage a2 and a4
        if (compute) {
            for (int i = tid; i < Bc * R; i += kCompute) {
                const int b = i / R, j = i - b * R;
                xa[b * RA + j] = fmaf(wi0[j], xprev[b], cur[b * PP + j]);
            }
            for (int i = tid; i < Bc * A; i += kCompute) {
                const int b = i / A, j = i - b * A;
                xa[b * RA + R + j] = cur[b * PP + R + j];               // a2
                fa[b * FA + F + j] = cur[b * PP + R + 2 * A + j];       // a4
            }
        }
        bar();

        // S2: h1 = GRUCell1(x, h1) for owned units → publish      (fatchord_version.py:210)
        if (compute)
            for (int it = it0; it < Bc * Uv; it += kWaves) {
                const int b = it / Uv, u = it - b * Uv, j = w * a.U + u;
                const float hn = gru_unit(S, a.s.wih1, a.s.whh1, a.s.bih1, a.s.bhh1, a.U, u, xa + b * RA, R,
                                          h1 + b * R, R, h1[b * R + j], lane);
                if (lane == 0) publish(xgH1 + b * R + j, tag, hn);
            }
        bar();   // all reads of h1(t-1) done before the gather overwrites it
        if (poller) gather(xgH1, Bc * R, R, h1, R, tag, a.ctl, a.timeout_ticks, t, HOP_H1, abort_flag);
        bar();
        if (*abort_flag) return;

        // S3: x = x + h1                                             (:212)
        if (compute)
            for (int i = tid; i < Bc * R; i += kCompute) {
                const int b = i / R, j = i - b * R;
                xa[b * RA + j] = xa[b * RA + j] + h1[i];
            }
        bar();

        // S4: h2 = GRUCell2([x; a2], h2) for owned units → publish (:213-214)
        if (compute)
            for (int it = it0; it < Bc * Uv; it += kWaves) {
                const int b = it / Uv, u = it - b * Uv, j = w * a.U + u;
                const float hn = gru_unit(S, a.s.wih2, a.s.whh2, a.s.bih2, a.s.bhh2, a.U, u, xa + b * RA, RA,
                                          h2 + b * R, R, h2[b * R + j], lane);
                if (lane == 0) publish(xgH2 + b * R + j, tag, hn);
            }
        bar();
        if (poller) gather(xgH2, Bc * R, R, h2, R, tag, a.ctl, a.timeout_ticks, t, HOP_H2, abort_flag);
        bar();
        if (*abort_flag) return;

        // S5: x = x + h2; stage a3                                    (:216-217)
        if (compute) {
            for (int i = tid; i < Bc * R; i += kCompute) {
                const int b = i / R, j = i - b * R;
                xa[b * RA + j] = xa[b * RA + j] + h2[i];
            }
            for (int i = tid; i < Bc * A; i += kCompute) {
                const int b = i / A, j = i - b * A;
                xa[b * RA + R + j] = cur[b * PP + R + A + j];
            }
        }
        bar();

        // S6: f1 = relu(fc1([x; a3])) owned rows → publish           (:217-218)
        if (compute)
            for (int it = it0; it < Bc * UFv; it += kWaves) {
                const int b = it / UFv, r = it - b * UFv, j = w * a.UF + r;
                float acc[1] = {0.f};
                dots<1>(S + a.s.w1 + r * RA, 0, xa + b * RA, RA / 4, lane, acc);
                const float v = wave_sum(acc[0]) + S[a.s.b1 + r];
                if (lane == 0) publish(xgF1 + b * F + j, tag, v > 0.0f ? v : 0.0f);
            }
        if (poller) gather(xgF1, Bc * F, F, fa, FA, tag, a.ctl, a.timeout_ticks, t, HOP_F1, abort_flag);
        bar();
        if (*abort_flag) return;

        // S7: f2 = relu(fc2([f1; a4])) owned rows → publish          (:220-221)
        if (compute)
            for (int it = it0; it < Bc * UFv; it += kWaves) {
                const int b = it / UFv, r = it - b * UFv, j = w * a.UF + r;
                float acc[1] = {0.f};
                dots<1>(S + a.s.w2 + r * FA, 0, fa + b * FA, FA / 4, lane, acc);
                const float v = wave_sum(acc[0]) + S[a.s.b2 + r];
                if (lane == 0) publish(xgF2 + b * F + j, tag, v > 0.0f ? v : 0.0f);
            }
        if (poller) gather(xgF2, Bc * F, F, f2, F, tag, a.ctl, a.timeout_ticks, t, HOP_F2, abort_flag);
        bar();
        if (*abort_flag) return;

        // S8: logits = fc3(f2)                                        (:223)
        if (a.mol) {
            // all 30 rows redundantly in every workgroup (bit-identical everywhere)
            const int NC = a.NC;
            if (compute)
                for (int it = wave; it < Bc * NC; it += kWaves) {
                    const int b = it / NC, c = it - b * NC;
                    float acc[1] = {0.f};
                    dots<1>(S + a.s.w3 + c * F, 0, f2 + b * F, F / 4, lane, acc);
                    const float v = wave_sum(acc[0]) + S[a.s.b3 + c];
                    if (lane == 0) lg[b * ll.ncp + c] = v;
                }
        } else {
            if (compute)
                for (int it = it0; it < Bc * UCv; it += kWaves) {
                    const int b = it / UCv, r = it - b * UCv, j = w * a.UC + r;
                    float acc[1] = {0.f};
                    dots<1>(S + a.s.w3 + r * F, 0, f2 + b * F, F / 4, lane, acc);
                    const float v = wave_sum(acc[0]) + S[a.s.b3 + r];
                    if (lane == 0) publish(xgLG + b * a.NC + j, tag, v);
                }
            if (poller)
                gather(xgLG, Bc * a.NC, a.NC, lg, ll.ncp, tag, a.ctl, a.timeout_ticks, t, HOP_LOGITS, abort_flag);
        }
        bar();
        if (*abort_flag) return;

        // S9: sample one row per wave → x_t                          (:225-237)
        if (compute)
            for (int b = it0; b < Bc; b += kWaves) {
                const float *l = lg + b * ll.ncp;
                const float *u = cur + b * PP + R + 3 * A;               // this step's noise
                float x;
                int label = 0;
                if (a.mol) {
                    // utils/distribution.py:87-123
                    float v = -INFINITY;
                    if (lane < 10) v = l[lane] - logf(-logf(u[lane]));
                    int k = 0;
                    float best = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
#pragma unroll
                    for (int j = 1; j < 10; ++j) {
                        const float vj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
                        if (vj > best) { best = vj; k = j; }
                    }
                    const float mean = l[10 + k];
                    const float ls = fmaxf(l[20 + k], -32.23619130191664f);
                    const float u2 = u[10];
                    x = mean + expf(ls) * (logf(u2) - logf(1.0f - u2));
                    x = x < -1.0f ? -1.0f : x;
                    x = x > 1.0f ? 1.0f : x;
                } else {
                    // softmax → Categorical renormalise → argmax(p / q)
                    const int NC = a.NC;
                    float e[kClsPerLaneMax];
                    float m = -INFINITY;
#pragma unroll
                    for (int k = 0; k < kClsPerLaneMax; ++k) {
                        const int c = lane + 64 * k;
                        e[k] = (c < NC) ? l[c] : -INFINITY;
                        m = fmaxf(m, e[k]);
                    }
                    m = wave_max(m);
                    float s = 0.0f;
#pragma unroll
                    for (int k = 0; k < kClsPerLaneMax; ++k) {
                        const int c = lane + 64 * k;
                        e[k] = (c < NC) ? expf(e[k] - m) : 0.0f;
                        s += e[k];
                    }
                    s = wave_sum(s);
                    float s2 = 0.0f;
#pragma unroll
                    for (int k = 0; k < kClsPerLaneMax; ++k) {
                        e[k] = e[k] / s;
                        s2 += e[k];
                    }
                    s2 = wave_sum(s2);
                    float bv = -INFINITY;
                    int bi = 0x7FFFFFFF;
#pragma unroll
                    for (int k = 0; k < kClsPerLaneMax; ++k) {
                        const int c = lane + 64 * k;
                        if (c < NC) am_merge(bv, bi, (e[k] / s2) / u[c], c);
                    }
                    label = wave_argmax(bv, bi);
                    x = (2.0f * (float)label) / ((float)NC - 1.0f) - 1.0f;
                }
                if (lane == 0) { xprev[b] = x; lbl[b] = label; }
            }

        // loader: its DMA for step t+1 must have landed before the end-of-step barrier
        if (loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
    }
    if (writer && a.L > 0) {
        const size_t o = (size_t)(a.b0 + lane) * a.L + (a.L - 1);
        a.out[o] = xprev[lane];
        if (a.labels) a.labels[o] = lbl[lane];
    }
}

// --------------------------------------------------------- I-layer conditioning GEMM
// cI[t][b][r] = I.bias[r] + Σ_k I.weight[r][1+k] · cond[t][b0+b][k],  k < feat + aux
// (the conditioning columns of fatchord_version.py:208-209; the x_{t-1} column is applied
// inside the loop).  64×64 output tile per 256-thread block, K staged by 32.
__global__ __launch_bounds__(256) void ci_gemm_kernel(const float *__restrict__ cond, int CD, int Bt, int b0,
                                                      int Bc, int M, const float *__restrict__ W, int ldw,
                                                      const float *__restrict__ bias, int N, int K,
                                                      float *__restrict__ cI) {
    __shared__ float As[32][64 + 1];
    __shared__ float Ws[32][64 + 1];
    const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += 32) {
        for (int i = threadIdx.x; i < 64 * 32; i += 256) {
            const int mm = i >> 5, kk = i & 31, m = m0 + mm, k = k0 + kk;
            float v = 0.0f;
            if (m < M && k < K) {
                const int t = m / Bc, b = m - t * Bc;
                v = cond[((size_t)t * Bt + b0 + b) * CD + k];
            }
            As[kk][mm] = v;
            const int n = n0 + mm;
            Ws[kk][mm] = (n < N && k < K) ? W[(size_t)n * ldw + 1 + k] : 0.0f;
        }
        __syncthreads();
#pragma unroll 8
        for (int kk = 0; kk < 32; ++kk) {
            float av[4], wv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) { av[i] = As[kk][ty * 4 + i]; wv[i] = Ws[kk][tx * 4 + i]; }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], wv[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ty * 4 + i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tx * 4 + j;
            if (n < N) cI[(size_t)m * N + n] = acc[i][j] + bias[n];
        }
    }
}

// ------------------------------------------------------------------------ host launchers
hipError_t launch_ci_gemm(const float *cond, int CD, int Bt, int b0, int Bc, int L, const float *W, int ldw,
                          const float *bias, int N, int K, float *cI, hipStream_t st) {
    const int M = L * Bc;
    dim3 grid((M + 63) / 64, (N + 63) / 64);
    hipLaunchKernelGGL(ci_gemm_kernel, grid, dim3(256), 0, st, cond, CD, Bt, b0, Bc, M, W, ldw, bias, N, K, cI);
    return hipGetLastError();
}

hipError_t launch_loop(const LoopArgs &a, size_t lds_bytes, hipStream_t st) {
    hipLaunchKernelGGL(fatchord_loop_kernel, dim3(a.G), dim3(kThreads), lds_bytes, st, a);
    return hipGetLastError();
}

hipError_t prepare_loop_kernel(int max_lds_bytes) {
    return hipFuncSetAttribute((const void *)fatchord_loop_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               max_lds_bytes);
}

hipError_t loop_occupancy(int *blocks_per_cu, size_t lds_bytes) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fatchord_loop_kernel, kThreads, lds_bytes);
}

}  // namespace wrnn
