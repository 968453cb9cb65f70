// deepmind_xcd.hip — XCD-resident persistent kernel for the dual coarse/fine softmax WaveRNN
// (models/deepmind_version.py:75-165, hidden 896, quantisation 256): up to 4 rows per XCD, 32 per
// launch (BASELINE config 5: 32 utterances per GPU = one launch).
//
// The loop's 12.2 MB of fp32 weights are held once per XCD as MFMA A operands in the 32 CUs'
// registers and LDS (deepmind_xcd.h, DxA: 378 per lane and wave: 252 in AGPRs, 84 in VGPRs, 42
// in LDS); the 4 rows of an
// XCD are the batch columns of v_mfma_f32_4x4x1_16b_f32.  Every hand-off is an XCD-local granule
// vector ({tag = step + 1, value}, plain stores, 16-byte sc1 polls) as in fatchord_xcd.hip.
//
// Per step t (prev = the labels of step t − 1 of every row):
//   coarse gates of the own 14 units × 4 rows (R·h_{t-1} from the LDS partials, I_coarse(prev))
//                                                                       → publish h_c    [hop Hc]
//   h_c slice → O1 (1 set)  → barrier → relu(+b)                        → publish o1     [hop O1]
//   R[:, :S]·h_c — the coarse half of the next step's R·h (5 sets + a quarter set, accumulators
//   kept in registers), the o1 poll riding along
//   o1 slice → O2 (8 rows) → barrier → +b                               → publish logits [hop Lc]
//   sample c_t: wave n polls row n's 256 logits and samples it in every workgroup — no label
//   hop: softmax → Categorical ≡ argmax_c p_c / q_c, q ~ Exp(1) (the reference's multinomial
//   draw under the noise contract), taken as argmax_c l_c − log q_c (no exp, no divisions)
//   fine gates (R·h_{t-1}, I_fine(prev, c_t))                            → publish h_f    [hop Hf]
//   h_f slice → O3 → barrier → relu(+b)                                  → publish o3     [hop O3]
//   R[:, S:]·h_f (finishes R·h_t; partials → LDS for step t + 1), the o3 poll riding along
//   o3 slice → O4 → barrier → +b                                         → publish logits [hop Lf]
//   sample f_t; workgroup 0 of the XCD writes combine_signal(c_t, f_t) (utils/dsp.py:33)
// The draws of step t + 1 (Exp(1): injected, or Philox precomputed by philox_fill_kernel) are
// loaded into registers of waves 1..3 after the h_c poll; their logs go into an LDS ring while
// wave 0 publishes o1.
//
// Membership as in fatchord_xcd.hip (XCC id + per-XCD arrival counter; bounded waits).  fp32,
// sums re-associated; the sampled labels are checked bit-exact against the oracle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "deepmind_xcd.h"
#include "mfma_device.h"
#include "wrnn_device.h"
#include "xcd_device.h"

#ifndef WRNN_DX_GATE_WAVE
#define WRNN_DX_GATE_WAVE 0   // the wave whose lanes run the coarse / fine gates (3: A/B, slower)
#endif
// hop publishes as plain buffer stores through one wave-uniform descriptor + a 32-bit granule
// index (as fatchord_xcd.hip's xpub_b) instead of workgroup-scope atomic stores (global_store sc0)
// through 64-bit per-lane addresses
#ifndef WRNN_DX_PUB_BUF
#define WRNN_DX_PUB_BUF 1
#endif
// R·h group B (WG-local rows 48..83) of h_t in two places: its coarse half (h_c(t) columns) in step
// t's h_f hop window, the accumulators parked in LDS, its fine half at the start of step t + 1 —
// one MFMA chain as before (bit-identical sums).  0: both halves at the start of step t + 1, in
// the h_c hop window (round 5), where the MFMA stream ahead of the h_c poll delayed it.  (Measured
// in round 6 and not kept: the gate wave's coarse half in the coarse-logits window, and the fine
// half behind group A's in the o3 window — DESIGN.md §4.3a.)
#ifndef WRNN_DX_GB_SPLIT
#define WRNN_DX_GB_SPLIT 1
#endif
// diagnostics (timing only, wrong results): 1 = R·h group B after the h_c poll instead of in its
// window; 2 = the gate wave skips its share of group B; 3 / 4 = its coarse half skipped by the
// non-gate waves / by every wave
#ifndef WRNN_DX_GB_AFTER_POLL
#define WRNN_DX_GB_AFTER_POLL 0
#endif
#ifndef WRNN_DX_ORDERED_ARGMAX
#define WRNN_DX_ORDERED_ARGMAX 1   // samplers: lane l holds classes 4l..4l+3, value-only max + ballot
#endif

namespace wrnn {

namespace {

__device__ __forceinline__ f2v lds2(const float *p) { return *reinterpret_cast<const f2v *>(p); }
// log q of the Exp(1) draws (q ≥ 2^-24, normal): v_log_f32 (log2) · ln 2, monotone — the argmax
// it feeds only compares l_c − log q_c across classes
__device__ __forceinline__ float fast_log(float q) { return __builtin_amdgcn_logf(q) * 0.693147180559945309f; }
__device__ __forceinline__ f4v log4(f4v q) { return f4v{fast_log(q.x), fast_log(q.y), fast_log(q.z), fast_log(q.w)}; }

// wave w's slice of a 448-wide hop vector, 4 rows: columns 112w .. 112w + 111 = the 14 units of
// workgroups 8w .. 8w + 7.  Padded rows (WRNN_DX_PAD): 256 granule pairs, pair p = lane + 64i:
// row p / 64, workgroup 8w + (p % 64) / 8, units 2((p % 64) % 8) + {0, 1} (pair 7 of a workgroup
// = its two pads).  Unpadded: 224 pairs, p = min(lane + 64i, 223) (lanes 32..63 of i = 3 repeat
// pairs 192..223): row p / 56, columns 112w + 2(p % 56) + {0, 1}.
__device__ __forceinline__ int dx_pair(int lane, int i) {
    const int p = lane + 64 * i;
    if constexpr (WRNN_DX_PAD) return p;
    return p < 224 ? p : p - 32;
}
__device__ __forceinline__ int dx_poll_off(int w, int p) {   // bytes
    if constexpr (WRNN_DX_PAD) {
        const int n = p >> 6, q = p & 63;
        return (n * kDxSP + kDxUP * 8 * w + 2 * q) * 8;
    }
    const int n = p / 56, cp = p - 56 * n;
    return (n * kDxS + kDxKW * w + 2 * cp) * 8;
}

// bounded poll of the wave's slice into v (all granules tagged `tag` on return, or *lds_abort)
__device__ __forceinline__ void dx_poll(__amdgpu_buffer_rsrc_t r, int w, uint32_t tag, int *ctl, long long timeout,
                                        int step, int hop, int *lds_abort, int lane, u4v (&v)[4]) {
    const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (;;) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ld16_sc1(r, dx_poll_off(w, dx_pair(lane, i)));
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 4; ++i) ok &= (v[i].y == tag) & (v[i].w == tag);
        if (__ballot(!ok) == 0) return;
        if ((++spins & 63u) == 0) {
            const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > timeout;
            const bool other = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (late || other) {
                if (late) record_abort(ctl, -4, step, hop, blockIdx.x);
                *lds_abort = 1;
                return;
            }
        }
    }
}

// polled pairs → the wave's staging rows [n][kDxST] (column 2·pair within the row's 112; the
// padded form skips each workgroup's pad pair)
__device__ __forceinline__ void dx_stage(float *stg, int lane, const u4v (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int p = dx_pair(lane, i);
        int n, col;
        if constexpr (WRNN_DX_PAD) {
            const int q = p & 63;
            n = p >> 6;
            col = 14 * (q >> 3) + 2 * (q & 7);
            if ((q & 7) == 7) continue;   // pads
        } else {
            n = p / 56;
            col = 2 * (p - 56 * n);
        }
        *reinterpret_cast<f2v *>(stg + n * kDxST + col) = f2v{__uint_as_float(v[i].x), __uint_as_float(v[i].z)};
    }
}

// no poll riding along
struct MPollNoneDx {
    __device__ __forceinline__ void step(int) {}
};

// A poll that rides along an MFMA layer: loads issued at chunk kAt, checked after the layer
// (fallback: the bounded blocking poll), as MPoll in fatchord_xcdm.hip
template <int kAt>
struct DxRide {
    u4v v[4];
    __amdgpu_buffer_rsrc_t r;
    int w, lane;
    uint32_t tag;
    __device__ __forceinline__ DxRide(const unsigned long long *vec, int w_, uint32_t tag_, int lane_)
        : r(hop_rsrc(vec)), w(w_), lane(lane_), tag(tag_) {}
    __device__ __forceinline__ void step(int c) {
        if (c == kAt) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = ld16_sc1(r, dx_poll_off(w, dx_pair(lane, i)));
        }
    }
    __device__ __forceinline__ void finish(int *ctl, long long timeout, int step_, int hop, int *lds_abort) {
        // pinned after the layer (empty volatile asm, ordered with the MFMA asm): hipcc otherwise
        // hoists the tag test and its s_waitcnt into the layer's MFMA stream
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(v[i]));
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 4; ++i) ok &= (v[i].y == tag) & (v[i].w == tag);
        if (__ballot(!ok) != 0) dx_poll(r, w, tag, ctl, timeout, step_, hop, lds_abort, lane, v);
    }
};

// O1 / O3: one 16-row set (4 row groups × 4 k-slices) over the wave's 112 columns, 28 MFMAs in
// 4 accumulator chains; partials → P[wave][row 16][n (+1 pad)][k-slice 4] (row stride 20)
template <bool kAgpr>
__device__ __forceinline__ void dx_o13(const float (&A)[28], const float *stg, float *P, int lane, int wave) {
    const int j = lane & 3, g = (lane >> 2) & 3, sp = lane >> 4;
    const float *bp = stg + j * kDxST + 28 * sp;
    f4v acc[4], b[2];
    b[0] = lds4(bp);
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        if (c + 1 < 7) b[(c + 1) & 1] = lds4(bp + 4 * (c + 1));
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const int m = 4 * c + mm;
            if (m < 4) mfma_first<kAgpr>(acc[m & 3], A[m], b[c & 1][mm]);
            else mfma_acc<kAgpr>(acc[m & 3], A[m], b[c & 1][mm]);
        }
    }
    mfma_drain_begin();
#pragma unroll
    for (int q = 0; q < 4; ++q) mfma_tie(acc[q]);
    const f4v d = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    float *p = P + (wave * 16 + 4 * g) * 20 + 4 * j + sp;
    p[0] = d.x;
    p[20] = d.y;
    p[40] = d.z;
    p[60] = d.w;
}

// O2 / O4: 8 rows (2 row groups × 8 k-slices of 14 columns), 14 MFMAs in 4 chains; partials →
// P[wave][row 8][n 4][k-slice 8]
// (A operands from LDS: Al = the wave's [14][64] image)
__device__ __forceinline__ void dx_o24(const float *Al, const float *stg, float *P, int lane, int wave) {
    const int j = lane & 3, b = lane >> 2, g = b & 1, ks = b >> 1;
    const float *bp = stg + j * kDxST + 14 * ks;
    f4v acc[4];
    f2v x[7];
    float A[14];
#pragma unroll
    for (int m = 0; m < 14; ++m) A[m] = Al[m * 64 + lane];
#pragma unroll
    for (int c = 0; c < 7; ++c) x[c] = lds2(bp + 2 * c);
#pragma unroll
    for (int m = 0; m < 14; ++m) {
        if (m < 4) mfma_first<false>(acc[m & 3], A[m], x[m >> 1][m & 1]);
        else mfma_acc<false>(acc[m & 3], A[m], x[m >> 1][m & 1]);
    }
    mfma_drain_begin();
#pragma unroll
    for (int q = 0; q < 4; ++q) mfma_tie(acc[q]);
    const f4v d = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    float *p = P + ((wave * 8 + 4 * g) * 4 + j) * 8 + ks;
    p[0] = d.x;
    p[32] = d.y;
    p[64] = d.z;
    p[96] = d.w;
}

// One half (kHalf 0: coarse columns from h_c, 1: fine columns from h_f) of R·h over the wave's
// 112 columns for the sets [S0, S1) (sets 0..3 AGPR, set 4 VGPR; 28 MFMAs each) and, with kQ,
// the quarter set's 7 (A from LDS); one chain per set continued across the halves; hook.step(c)
// at each of the 7 chunks.  Two row groups run in different windows of the step (below): sets
// 0..2 (WG-local rows 0..47: every coarse gate row) and sets 3, 4 + the quarter (rows 48..83).
template <int kHalf, int S0, int S1, bool kQ, typename Hook>
__device__ __forceinline__ void dx_rhalf(const float (&AR)[5][56], const float *ARQl, const float *stg,
                                         f4v (&accR)[5], f4v &accQ, int lane, Hook &hook) {
    const int j = lane & 3, sp = lane >> 4, b = lane >> 2;
    const float *bp = stg + j * kDxST + 28 * sp;
    const float *bq = stg + j * kDxST + 7 * b;
    f4v bb[2];
    bb[0] = lds4(bp);
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        hook.step(c);
        if (c + 1 < 7) bb[(c + 1) & 1] = lds4(bp + 4 * (c + 1));
        float qv = 0.0f, qa = 0.0f;
        if constexpr (kQ) {
            qv = bq[c];
            qa = ARQl[(7 * kHalf + c) * 64 + lane];
        }
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const int m = 4 * c + mm;
#pragma unroll
            for (int s = S0; s < S1; ++s) {
                const float a = AR[s][28 * kHalf + m], x = bb[c & 1][mm];
                if (kHalf == 0 && m == 0) {
                    if (s < 4) mfma_first<true>(accR[s], a, x);
                    else mfma_first<false>(accR[s], a, x);
                } else {
                    if (s < 4) mfma_acc<true>(accR[s], a, x);
                    else mfma_acc<false>(accR[s], a, x);
                }
            }
        }
        if constexpr (kQ) {
            if (kHalf == 0 && c == 0) mfma_first<false>(accQ, qa, qv);
            else mfma_acc<false>(accQ, qa, qv);
        }
    }
}

// R·h partials of the sets [S0, S1) (+ the quarter set) → LDS: sets [set][wave][row 16][n (+1)][k-slice 4],
// quarter [wave][row 4][n][16]
template <int S0, int S1, bool kQ>
__device__ __forceinline__ void dx_rput(f4v (&accR)[5], f4v &accQ, float *PR, float *PRQ, int lane, int wave) {
    mfma_drain_begin();
#pragma unroll
    for (int s = S0; s < S1; ++s) mfma_tie(accR[s]);
    if constexpr (kQ) mfma_tie(accQ);
    const int j = lane & 3, g = (lane >> 2) & 3, sp = lane >> 4, b = lane >> 2;
#pragma unroll
    for (int s = S0; s < S1; ++s) {
        float *p = PR + ((s * kDxWaves + wave) * 16 + 4 * g) * 20 + 4 * j + sp;
        p[0] = accR[s].x;
        p[20] = accR[s].y;
        p[40] = accR[s].z;
        p[60] = accR[s].w;
    }
    if constexpr (kQ) {
        float *q = PRQ + (wave * 16 + j) * 16 + b;   // [wave][row i][n j][slice b]: row stride 64
        q[0] = accQ.x;
        q[64] = accQ.y;
        q[128] = accQ.z;
        q[192] = accQ.w;
    }
}

// Σ over waves and k-slices of WG-local R row rr (0..83), batch row n — fixed order
__device__ __forceinline__ float dx_rsum(const float *PR, const float *PRQ, int rr, int n) {
    float t[kDxWaves];
    if (rr < 80) {
        const int s = rr >> 4, r = rr & 15;
#pragma unroll
        for (int w = 0; w < kDxWaves; ++w) {
            const f4v u = lds4(PR + ((s * kDxWaves + w) * 16 + r) * 20 + 4 * n);
            t[w] = (u.x + u.y) + (u.z + u.w);
        }
    } else {
        const int i = rr - 80;
#pragma unroll
        for (int w = 0; w < kDxWaves; ++w) {
            const float *p = PRQ + ((w * 4 + i) * 4 + n) * 16;
            const f4v u0 = lds4(p), u1 = lds4(p + 4), u2 = lds4(p + 8), u3 = lds4(p + 12);
            t[w] = (((u0.x + u0.y) + (u0.z + u0.w)) + ((u1.x + u1.y) + (u1.z + u1.w))) +
                   (((u2.x + u2.y) + (u2.z + u2.w)) + ((u3.x + u3.y) + (u3.z + u3.w)));
        }
    }
    return (t[0] + t[1]) + (t[2] + t[3]);
}

// Σ of an O1 / O3 output (row r < 16, n) and of an O2 / O4 output (row r < 8, n)
// (all partial loads issued before the first add — a scheduling barrier between them: hipcc
// otherwise interleaves reads and adds two loads at a time, one LDS round trip per pair)
__device__ __forceinline__ float dx_o13sum(const float *P, int r, int n) {
    f4v u[kDxWaves];
#pragma unroll
    for (int w = 0; w < kDxWaves; ++w) u[w] = lds4(P + (w * 16 + r) * 20 + 4 * n);
    __builtin_amdgcn_sched_barrier(0);
    float t[kDxWaves];
#pragma unroll
    for (int w = 0; w < kDxWaves; ++w) t[w] = (u[w].x + u[w].y) + (u[w].z + u[w].w);
    return (t[0] + t[1]) + (t[2] + t[3]);
}
__device__ __forceinline__ float dx_o24sum(const float *P, int r, int n) {
    f4v u0[kDxWaves], u1[kDxWaves];
#pragma unroll
    for (int w = 0; w < kDxWaves; ++w) {
        const float *p = P + ((w * 8 + r) * 4 + n) * 8;
        u0[w] = lds4(p);
        u1[w] = lds4(p + 4);
    }
    __builtin_amdgcn_sched_barrier(0);
    float t[kDxWaves];
#pragma unroll
    for (int w = 0; w < kDxWaves; ++w)
        t[w] = ((u0[w].x + u0[w].y) + (u0[w].z + u0[w].w)) + ((u1[w].x + u1[w].y) + (u1[w].z + u1[w].w));
    return (t[0] + t[1]) + (t[2] + t[3]);
}

}  // namespace

#define DSTR(kk)                                                                                             \
    do {                                                                                                     \
        if (kDbg && lane == 0 && (unsigned)(t - a.t0 - kDxDbgSkip) < (unsigned)kDxDbgSteps)                 \
            dbgs[((t - a.t0 - kDxDbgSkip) * kDxWaves + wave) * kDxStamps + (kk)] =                           \
                (unsigned)__builtin_amdgcn_s_memrealtime();                                                  \
    } while (0)
#define DST(kk)                                                                                              \
    do {                                                                                                     \
        if (kDbg && lane == 0 && (unsigned)(t - a.t0 - kDxDbgSkip) < (unsigned)kDxDbgSteps)                 \
            dbgs[((t - a.t0 - kDxDbgSkip) * kDxWaves + wave) * kDxStamps + (kk)] =                           \
                (unsigned)__builtin_amdgcn_s_memtime();                                                      \
    } while (0)

template <bool kDbg>
__global__ __launch_bounds__(kDxThreads, 1) void deepmind_xcd_kernel(DxArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const DxLds ll = dx_lds_layout(kDbg);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    float *pr = smem + ll.pr, *prq = smem + ll.prq, *po1 = smem + ll.po1, *po3 = smem + ll.po3;
    float *po2 = smem + ll.po2, *po4 = smem + ll.po4, *nzr = smem + ll.nz;
    float *cst = smem + ll.cst, *lab = smem + ll.lab, *rs = smem + ll.rs;
    int *misc = reinterpret_cast<int *>(smem + ll.misc);
    int *abort_flag = misc;
    unsigned *dbgs = reinterpret_cast<unsigned *>(smem + ll.dbg);
    auto stg_of = [&](int vec) { return smem + ll.stg + (vec * kDxWaves + wave) * 4 * kDxST; };
    float *aol = smem + ll.ao + wave * kDxAL * 64;   // this wave's LDS A operands
    const float *arq = aol, *ao2 = aol + 14 * 64, *ao4 = aol + 28 * 64;

    // ---- membership: XCD k (launch rows k, k + 8, k + 16, k + 24) and index c within it
    if (tid == 0) {
        const int kx = (int)xcc_id();
        int cc = kXcdWgs;
        if (kx < a.nb) cc = atomicAdd(&a.members[kx], 1);
        misc[1] = (kx < a.nb && cc < kXcdWgs) ? kx * kXcdWgs + cc : -1;
        misc[0] = 0;
    }
    __syncthreads();
    const int mem = __builtin_amdgcn_readfirstlane(misc[1]);   // wave-uniform: hop addresses in SGPRs
    if (mem < 0) return;
    const int k = mem / kXcdWgs, c = mem - k * kXcdWgs;
    const int RX = min(kDxRowsXcd, (a.nb - k + kXcds - 1) / kXcds);   // rows n < RX: launch row k + 8n
    unsigned long long *xg = a.xg + (size_t)k * kDxXcdStride;
    const __amdgpu_buffer_rsrc_t xgr = __builtin_amdgcn_make_buffer_rsrc(xg, 0, 0x7fffffff, 0x00020000);
    // publish granule `gi` (index into the XCD's hop area) of this step
    auto pub = [&](int gi, uint32_t tg, float v) {
        if (WRNN_DX_PUB_BUF) xpub_b(xgr, gi, tg, v);
        else xpub(xg + gi, tg, v);
    };
    const float *S = a.slab + (size_t)(k * kXcdWgs + c) * a.s.total;

    // ---- register-resident A operands
    float AR[5][56], AO1[28], AO3[28];
    {
        const float *Aw = S + a.s.a + (size_t)wave * kDxA * 64 + lane;
#pragma unroll
        for (int s = 0; s < 5; ++s)
#pragma unroll
            for (int m = 0; m < 56; ++m) AR[s][m] = Aw[(DA_R + 56 * s + m) * 64];
#pragma unroll
        for (int m = 0; m < 28; ++m) {
            AO1[m] = Aw[(DA_O1 + m) * 64];
            AO3[m] = Aw[(DA_O3 + m) * 64];
        }
        // the quarter set and O2 / O4 → LDS
        for (int m = 0; m < kDxAL; ++m) aol[m * 64 + lane] = Aw[(DA_RQ + m) * 64];
    }

    // roles: gate threads (unit u, row n), 56 of them; O1/O3 epilogue (row r < 14, n); O2/O4 (r < 8, n)
    // the gate threads are lanes 0..55 of wave WRNN_DX_GATE_WAVE (wave 3 instead of 0, so that
    // wave 0's row-group-B share would not follow the gates: 6.63 → 6.68 µs/step at 32 rows,
    // profiles/r05_ab_dx_gate_wave.log)
    const bool gate = (tid >> 6) == WRNN_DX_GATE_WAVE && (tid & 63) < 4 * kDxU;
    const int gu = (tid & 63) % kDxU, gn = (tid & 63) / kDxU;
    const int t_end = a.t0 + a.Lc;
    float *st = a.state + (size_t)(k * kXcdWgs + c) * kDxStateW;
    auto noise_src = [&](int t, int n) {
        return a.noise + ((size_t)(t - a.nz_t0) * a.nz_ts + a.nz_b0 + k + kXcds * n) * (2 * kDxQ);
    };

    // ---- prologue: constants, carried state, draws of step t0
    for (int i = tid; i < kDxCst; i += kDxThreads) cst[i] = S[a.s.cst + i];
    const bool resume = a.t0 > 0;
    for (int i = tid; i < kDxPR; i += kDxThreads) pr[i] = resume ? st[8 * kDxU + i] : 0.0f;
    for (int i = tid; i < kDxPRQ; i += kDxThreads) prq[i] = resume ? st[8 * kDxU + kDxPR + i] : 0.0f;
    if (tid < 16) lab[tid] = (resume && tid < 8) ? st[8 * kDxU + kDxPR + kDxPRQ + tid] : 0.0f;   // out_coarse = out_fine = 0 (:89-90)
    // Σ R·h of every own gate row (WG-local row rr, batch row n) → rs[rr·4 + n], from the partials
    auto r_sums = [&](int e0, int de, int r0, int r1) {
        for (int e = r0 * 4 + e0; e < r1 * 4; e += de) rs[e] = dx_rsum(pr, prq, e >> 2, e & 3);
    };
    float hc = 0.0f, hf = 0.0f;   // h of (unit gu, row gn): this thread's recurrent state
    if (gate && resume) {
        hc = st[gn * 2 * kDxU + gu];
        hf = st[gn * 2 * kDxU + kDxU + gu];
    }
    // consume the carried-state loads here: left pending into the loop, the gates' first use of
    // hc waits on vmcnt inside every step (behind the wave's in-flight publishes)
    asm volatile("" : "+v"(hc), "+v"(hf));
    for (int i = tid; i < RX * 2 * kDxQ / 4; i += kDxThreads) {
        const int n = i / (2 * kDxQ / 4), f = i - n * (2 * kDxQ / 4);
        *reinterpret_cast<f4v *>(nzr + ((a.t0 & 1) * 4 + n) * 2 * kDxQ + 4 * f) =
            log4(*reinterpret_cast<const f4v *>(noise_src(a.t0, n) + 4 * f));
    }
    __syncthreads();
    r_sums(tid, kDxThreads, 0, 84);
    __syncthreads();

    // R[rows 48..83, :]·h of the staged h_c (stg_of(2)) and h_f (stg_of(0)) slices → partials
    float *gbc = smem + ll.gbc + wave * 3 * 4 * 64;   // this wave's parked group-B accumulators
    // the coarse half of group B of R·h_t (h_c(t) staged in stg_of(2)) → gbc
    auto r_group_b_coarse = [&]() {
        f4v bR[5], bQ;
        MPollNoneDx none;
        dx_rhalf<0, 3, 5, true>(AR, arq, stg_of(2), bR, bQ, lane, none);
        mfma_drain_begin();
        mfma_tie(bR[3]);
        mfma_tie(bR[4]);
        mfma_tie(bQ);
        *reinterpret_cast<f4v *>(gbc + (0 * 64 + lane) * 4) = bR[3];
        *reinterpret_cast<f4v *>(gbc + (1 * 64 + lane) * 4) = bR[4];
        *reinterpret_cast<f4v *>(gbc + (2 * 64 + lane) * 4) = bQ;
    };
    // its fine half (h_f(t) in stg_of(0)) continuing the parked chains → partials
    auto r_group_b_fine = [&]() {
        f4v bR[5], bQ;
        MPollNoneDx none;
        bR[3] = lds4(gbc + (0 * 64 + lane) * 4);
        bR[4] = lds4(gbc + (1 * 64 + lane) * 4);
        bQ = lds4(gbc + (2 * 64 + lane) * 4);
        dx_rhalf<1, 3, 5, true>(AR, arq, stg_of(0), bR, bQ, lane, none);
        dx_rput<3, 5, true>(bR, bQ, pr, prq, lane, wave);
    };
    auto r_group_b = [&]() {
        f4v bR[5], bQ;
        MPollNoneDx none;
        // (diagnostics 3 / 4: the coarse half skipped by the non-gate waves / by every wave)
        const bool skip_c = WRNN_DX_GB_AFTER_POLL == 4 || (WRNN_DX_GB_AFTER_POLL == 3 && wave != WRNN_DX_GATE_WAVE);
        if (skip_c) {
#pragma unroll
            for (int s = 0; s < 5; ++s) bR[s] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
            bQ = f4v{0.0f, 0.0f, 0.0f, 0.0f};
        } else {
            dx_rhalf<0, 3, 5, true>(AR, arq, stg_of(2), bR, bQ, lane, none);
        }
        dx_rhalf<1, 3, 5, true>(AR, arq, stg_of(0), bR, bQ, lane, none);
        dx_rput<3, 5, true>(bR, bQ, pr, prq, lane, wave);
    };

    constexpr int kNzF4 = 2 * kDxQ / 4;                         // float4s of one row's draws
    // draws loaded by waves 1..3 (wave 0 publishes the O1 epilogue meanwhile)
    constexpr int kNzThreads = kDxThreads - 64;
    constexpr int kNzLd = (kDxRowsXcd * kNzF4 + kNzThreads - 1) / kNzThreads;   // per thread

    for (int t = a.t0; t < t_end; ++t) {
        int tid = threadIdx.x;   // opaque per step (see fatchord_xcdm.hip)
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, gu = lane % kDxU, gn = lane / kDxU;
        const uint32_t tag = (uint32_t)t + 1u;
        const bool more = t + 1 < t_end;
        DST(0);
        if (kDbg && lane == 0 && (unsigned)(t - a.t0 - kDxDbgSkip) < (unsigned)kDxDbgSteps)
            dbgs[((t - a.t0 - kDxDbgSkip) * kDxWaves + wave) * kDxStamps + kDxStamps - 1] =
                (unsigned)__builtin_amdgcn_s_memrealtime();
        // the pads of this step's 448-wide hop rows (lanes 56..63 of wave 0: 4 rows × 2 per hop),
        // tagged like the data: every workgroup has finished polling step t − 1's vectors before
        // any workgroup starts step t (its logits came after those polls)
        // (measured in round 6: the pads written beside each hop's data, or for step t + 1 at the end
        // of step t, run no faster, profiles/r06_ab_dx_padlate.log)
        if (WRNN_DX_PAD && wave == 0 && lane >= 4 * kDxU) {
            const int pl = lane - 4 * kDxU;
            const int pad = (pl >> 1) * kDxSP + kDxUP * c + kDxU + (pl & 1);
            pub(pad + kDxHopOff[DX_HC], tag, 0.0f);
            pub(pad + kDxHopOff[DX_O1], tag, 0.0f);
            pub(pad + kDxHopOff[DX_HF], tag, 0.0f);
            pub(pad + kDxHopOff[DX_O3], tag, 0.0f);
        }
        // ---- coarse gates (:106-125): R·h_{t-1} (partials of the previous step), I_coarse(prev)
        if (gate) {
            // every LDS operand of the gate chain issued at once (one round trip: hipcc otherwise
            // waits on the labels before issuing the weight / sum / bias reads)
            const float l0 = lab[gn], l1 = lab[4 + gn];
            float w0[3], w1[3], Rg[3];
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const float *wi = cst + DC_IC + (g * kDxU + gu) * 2;
                w0[g] = wi[0];
                w1[g] = wi[1];
                Rg[g] = rs[(g * kDxU + gu) * 4 + gn];
            }
            const float bu = cst[DC_BU + gu], br = cst[DC_BR + gu], be = cst[DC_BE + gu];
            __builtin_amdgcn_sched_barrier(0);
            const float x0 = label_x(l0), x1 = label_x(l1);
            float I[3];
#pragma unroll
            for (int g = 0; g < 3; ++g) I[g] = __fadd_rn(__fmul_rn(w0[g], x0), __fmul_rn(w1[g], x1));   // separately rounded products (:111)
            const float uu = sigmoid_((Rg[0] + I[0]) + bu);
            const float rr = sigmoid_((Rg[1] + I[1]) + br);
            const float ee = tanh_((rr * Rg[2] + I[2]) + be);
            hc = uu * hc + (1.0f - uu) * ee;
            pub(kDxHopOff[DX_HC] + gn * kDxSP + kDxUP * c + gu, tag, hc);
            DST(19);
            DSTR(22);   // (s_memrealtime: the h_c hop measured across workgroups, tools/stamps_dx.py)
        }
        // row group B (WG-local rows 48..83: fine gate rows only) of R·h_{t-1}, both halves from the
        // still-staged h_c(t-1) / h_f(t-1) slices: the other waves while the gate wave runs the
        // coarse gates, the gate wave in its h_c hop wait; partials → LDS (summed in this step's O2
        // epilogue window)
        if ((WRNN_DX_GB_AFTER_POLL != 1 && (WRNN_DX_GB_AFTER_POLL != 2 || wave != WRNN_DX_GATE_WAVE)) && t > a.t0) {
            if (WRNN_DX_GB_SPLIT) r_group_b_fine();
            else r_group_b();
        }
        DST(1);
        // ---- h_c slice → O1 → relu → o1
        {
            u4v v[4];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            DST(20);
            dx_poll(hop_rsrc(xg + kDxHopOff[DX_HC]), wave, tag, a.ctl, a.timeout_ticks, t, DX_HC, abort_flag, lane, v);
            DSTR(21);
            dx_stage(stg_of(2), lane, v);
        }
        if (WRNN_DX_GB_AFTER_POLL == 1 && t > a.t0) r_group_b();
        // the draws of step t + 1 → registers of waves 1..3; their logs go into the ring while
        // wave 0 publishes o1 (below)
        f4v nzl[kNzLd];
        const int lt = tid - 64;
        if (more && lt >= 0) {
#pragma unroll
            for (int i = 0; i < kNzLd; ++i) {
                const int idx = lt + kNzThreads * i;
                if (idx < RX * kNzF4) {
                    const int n = idx / kNzF4, f = idx - n * kNzF4;
                    nzl[i] = *reinterpret_cast<const f4v *>(noise_src(t + 1, n) + 4 * f);
                }
            }
        }
        DST(2);
        // epilogue biases read before the layer (pinned: off the post-barrier LDS chain)
        float bo1 = cst[DC_B1 + tid % kDxU], bo2 = cst[DC_B2 + tid % kDxUO2];
        asm volatile("" : "+v"(bo1), "+v"(bo2));
        dx_o13<true>(AO1, stg_of(2), po1, lane, wave);
        bar();
        DST(3);
        if (tid < 4 * kDxU) {
            const int r = tid % kDxU, n = tid / kDxU;
            const float o = dx_o13sum(po1, r, n) + bo1;
            pub(kDxHopOff[DX_O1] + n * kDxSP + kDxUP * c + r, tag, o > 0.0f ? o : 0.0f);
        } else if (more && lt >= 0) {   // log q of step t + 1 → ring slot (t + 1) & 1
            float *slot = nzr + ((t + 1) & 1) * 4 * 2 * kDxQ;
#pragma unroll
            for (int i = 0; i < kNzLd; ++i) {
                const int idx = lt + kNzThreads * i;
                if (idx < RX * kNzF4) {
                    const int n = idx / kNzF4, f = idx - n * kNzF4;
                    *reinterpret_cast<f4v *>(slot + n * 2 * kDxQ + 4 * f) = log4(nzl[i]);
                }
            }
        }
        DST(4);
        // ---- R[rows 0..47, :S]·h_c (next step's R·h, coarse half of row group A) with the o1 poll
        // riding along; group B (rows 48..83) runs at the start of the next step
        f4v accR[5], accQ;
        {
            DxRide<4> po(xg + kDxHopOff[DX_O1], wave, tag, lane);
            dx_rhalf<0, 0, 3, false>(AR, arq, stg_of(2), accR, accQ, lane, po);
            DST(5);
            po.finish(a.ctl, a.timeout_ticks, t, DX_O1, abort_flag);
            dx_stage(stg_of(1), lane, po.v);
        }
        DST(6);
        // ---- o1 slice → O2 → coarse logits
        dx_o24(ao2, stg_of(1), po2, lane, wave);
        bar();
        DST(7);
        if (tid < 4 * kDxUO2) {
            const int r = tid % kDxUO2, n = tid / kDxUO2;
            pub(kDxHopOff[DX_LC] + n * kDxQ + kDxUO2 * c + r, tag, dx_o24sum(po2, r, n) + bo2);
        } else if (tid >= 64 && t > a.t0) {
            r_sums(tid - 64, kDxThreads - 64, 48, 84);   // group B of R·h_{t-1} (partials from this step's start)
        }
        DST(8);
        // ---- sample c_t (:129-131): wave n samples row n
        auto sample_row = [&](int hop, int half) -> int {
            const __amdgpu_buffer_rsrc_t rl = hop_rsrc(xg + kDxHopOff[hop]);
            // log q of this row's draws (written a step ahead) read before the logits poll: its
            // LDS round trip off the chain that follows the poll
            const float *lq = nzr + ((t & 1) * 4 + wave) * 2 * kDxQ + half * kDxQ;
            f4v q = lds4(lq + 4 * lane);
            asm volatile("" : "+v"(q));
            const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
            unsigned spins = 0;
            bool dead = false;
            u4v v0, v1;   // polled in place: the exit path is one uniform branch, no copies
            for (;;) {
                v0 = ld16_sc1(rl, (wave * kDxQ + (WRNN_DX_ORDERED_ARGMAX ? 4 * lane : 2 * lane)) * 8);
                v1 = ld16_sc1(rl, (wave * kDxQ + (WRNN_DX_ORDERED_ARGMAX ? 4 * lane + 2 : 2 * lane + 128)) * 8);
                const bool ok = (v0.y == tag) & (v0.w == tag) & (v1.y == tag) & (v1.w == tag);
                if (__ballot(!ok) == 0) break;
                if ((++spins & 63u) == 0) {
                    const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                    const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    if (late || other) {
                        if (late) record_abort(a.ctl, -4, t, hop, blockIdx.x);
                        *abort_flag = 1;
                        dead = true;
                        break;
                    }
                }
            }
            if (dead) return 0;
            const f4v lv = {__uint_as_float(v0.x), __uint_as_float(v0.z), __uint_as_float(v1.x), __uint_as_float(v1.z)};
            // argmax_c l_c − log q_c ≡ argmax_c p_c / q_c (softmax, Categorical renormalisation and
            // the draw's scale cancel): lane l holds classes 4l .. 4l + 3, so the winner is the first
            // lane holding the wave's max (wave_argmax_ordered: no index through the DPP stages)
            if constexpr (WRNN_DX_ORDERED_ARGMAX) {
                float bv = lv.x - q.x;
                int bi = 4 * lane;
                am_merge(bv, bi, lv.y - q.y, 4 * lane + 1);
                am_merge(bv, bi, lv.z - q.z, 4 * lane + 2);
                am_merge(bv, bi, lv.w - q.w, 4 * lane + 3);
                return wave_argmax_ordered(bv, bi);
            } else {   // (round 3: classes 2l, 2l + 1, 2l + 128, 2l + 129, index through the DPP stages)
                const f2v q0 = lds2(lq + 2 * lane), q1 = lds2(lq + 2 * lane + 128);
                float bv = lv.x - q0.x;
                int bi = 2 * lane;
                am_merge(bv, bi, lv.y - q0.y, 2 * lane + 1);
                am_merge(bv, bi, lv.z - q1.x, 2 * lane + 128);
                am_merge(bv, bi, lv.w - q1.y, 2 * lane + 129);
                return wave_argmax(bv, bi);
            }
        };
        if (wave < RX) {
            const int cl = sample_row(DX_LC, 0);
            if (lane == 0) lab[8 + wave] = (float)cl;
        }
        bar();
        DST(9);
        // ---- fine gates (:135-145): I_fine(prev, c_t)
        if (gate) {
            const float l0 = lab[gn], l1 = lab[4 + gn], l2 = lab[8 + gn];   // (all reads at once, as above)
            float w0[3], w1[3], w2[3], Rg[3];
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const float *wi = cst + DC_IF + (g * kDxU + gu) * 3;
                w0[g] = wi[0];
                w1[g] = wi[1];
                w2[g] = wi[2];
                Rg[g] = rs[((3 + g) * kDxU + gu) * 4 + gn];
            }
            const float bu = cst[DC_BU + kDxU + gu], br = cst[DC_BR + kDxU + gu], be = cst[DC_BE + kDxU + gu];
            __builtin_amdgcn_sched_barrier(0);
            const float x0 = label_x(l0), x1 = label_x(l1), x2 = label_x(l2);
            float I[3];
#pragma unroll
            for (int g = 0; g < 3; ++g)   // (:137)
                I[g] = __fadd_rn(__fadd_rn(__fmul_rn(w0[g], x0), __fmul_rn(w1[g], x1)), __fmul_rn(w2[g], x2));
            const float uu = sigmoid_((Rg[0] + I[0]) + bu);
            const float rr = sigmoid_((Rg[1] + I[1]) + br);
            const float ee = tanh_((rr * Rg[2] + I[2]) + be);
            hf = uu * hf + (1.0f - uu) * ee;
            pub(kDxHopOff[DX_HF] + gn * kDxSP + kDxUP * c + gu, tag, hf);
            DSTR(23);   // (the h_f hop in real time, as slots 22 / 21 for h_c)
        }
        // the coarse half of group B of R·h_t (the next step's fine half continues it): every wave
        // in the h_f hop window (waves 1..3 idle there; the gate wave after publishing h_f)
        if (WRNN_DX_GB_SPLIT && more) r_group_b_coarse();
        DST(10);
        // ---- h_f slice → O3 → relu → o3
        {
            u4v v[4];
            dx_poll(hop_rsrc(xg + kDxHopOff[DX_HF]), wave, tag, a.ctl, a.timeout_ticks, t, DX_HF, abort_flag, lane, v);
            DSTR(24);
            dx_stage(stg_of(0), lane, v);
        }
        DST(11);
        float bo3 = cst[DC_B3 + tid % kDxU], bo4 = cst[DC_B4 + tid % kDxUO2];
        asm volatile("" : "+v"(bo3), "+v"(bo4));
        dx_o13<false>(AO3, stg_of(0), po3, lane, wave);
        bar();
        DST(12);
        if (tid < 4 * kDxU) {
            const int r = tid % kDxU, n = tid / kDxU;
            const float o = dx_o13sum(po3, r, n) + bo3;
            pub(kDxHopOff[DX_O3] + n * kDxSP + kDxUP * c + r, tag, o > 0.0f ? o : 0.0f);
        }
        DST(13);
        // ---- R[rows 0..47, S:]·h_f finishes group A of R·h_t (the gates above have read R·h_{t-1})
        // → LDS partials
        {
            DxRide<4> po(xg + kDxHopOff[DX_O3], wave, tag, lane);
            dx_rhalf<1, 0, 3, false>(AR, arq, stg_of(0), accR, accQ, lane, po);
            dx_rput<0, 3, false>(accR, accQ, pr, prq, lane, wave);
            DST(14);
            po.finish(a.ctl, a.timeout_ticks, t, DX_O3, abort_flag);
            dx_stage(stg_of(1), lane, po.v);
        }
        DST(15);
        // ---- o3 slice → O4 → fine logits
        dx_o24(ao4, stg_of(1), po4, lane, wave);
        bar();
        DST(16);
        if (tid < 4 * kDxUO2) {
            const int r = tid % kDxUO2, n = tid / kDxUO2;
            pub(kDxHopOff[DX_LF] + n * kDxQ + kDxUO2 * c + r, tag, dx_o24sum(po4, r, n) + bo4);
        } else if (tid >= 64) {
            r_sums(tid - 64, kDxThreads - 64, 0, 48);   // group A of R·h_t (complete since the barrier)
        }
        DST(17);
        // ---- sample f_t (:149-151); combine_signal (utils/dsp.py:33); previous labels ← (c_t, f_t)
        if (wave < RX) {
            const int fl = sample_row(DX_LF, 1);
            if (lane == 0) {
                const float cl = lab[8 + wave];
                lab[wave] = cl;
                lab[4 + wave] = (float)fl;
                if (c == 0) {
                    const int v = (int)cl * 256 + fl - 32768;
                    const size_t o = (size_t)(a.b0 + k + kXcds * wave) * a.L + t;
                    a.out[o] = (float)v;
                    if (a.labels) a.labels[o] = v;
                }
            }
        }
        DST(18);
        bar();
        if (*abort_flag) return;
    }
    // row group B of the last step's R·h (the next chunk starts from complete partials)
    if (a.Lc > 0) r_group_b();
    __syncthreads();
    if (kDbg && a.dbg) {
        __syncthreads();
        for (int i = tid; i < kDxDbgSteps * kDxWaves * kDxStamps; i += kDxThreads) {
            const int stp = i / (kDxWaves * kDxStamps), w = (i / kDxStamps) % kDxWaves, kk = i % kDxStamps;
            a.dbg[(((size_t)blockIdx.x * kDxWaves + w) * kDxDbgSteps + stp) * kDxStamps + kk] = dbgs[i];
        }
    }
    // ---- carry the recurrent state to the next time chunk
    if (gate) {
        st[gn * 2 * kDxU + gu] = hc;
        st[gn * 2 * kDxU + kDxU + gu] = hf;
    }
    for (int i = tid; i < kDxPR; i += kDxThreads) st[8 * kDxU + i] = pr[i];
    for (int i = tid; i < kDxPRQ; i += kDxThreads) st[8 * kDxU + kDxPR + i] = prq[i];
    if (tid < 8) st[8 * kDxU + kDxPR + kDxPRQ + tid] = lab[tid];
}

hipError_t launch_dx(const DxArgs &a, hipStream_t st) {
    DxArgs args = a;
    void *params[] = {&args};
    const bool dbg = a.dbg != nullptr;
    const void *kf = dbg ? (const void *)deepmind_xcd_kernel<true> : (const void *)deepmind_xcd_kernel<false>;
    return hipLaunchKernel(kf, dim3(kXcds * kXcdWgs), dim3(kDxThreads), params, dx_lds_layout(dbg).total * sizeof(float),
                           st);
}

// set the LDS limit; *ok = the launch is co-resident (one workgroup per CU)
hipError_t prepare_dx_kernel(int max_lds_bytes, bool *ok) {
    *ok = false;
    for (int dbg = 0; dbg < 2; ++dbg) {
        const void *kf = dbg ? (const void *)deepmind_xcd_kernel<true> : (const void *)deepmind_xcd_kernel<false>;
        const size_t lds = dx_lds_layout(dbg).total * sizeof(float);
        if (lds > (size_t)max_lds_bytes) return hipSuccess;
        hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds_bytes);
        if (e != hipSuccess) return e;
        int n = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kf, kDxThreads, lds);
        if (e != hipSuccess) return e;
        if (n < 1) return hipSuccess;
    }
    *ok = true;
    return hipSuccess;
}

}  // namespace wrnn
