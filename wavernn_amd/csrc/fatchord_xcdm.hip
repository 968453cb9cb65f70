// fatchord_xcdm.hip — XCD-resident persistent kernel for MANY MoL rows (rnn 512, fc 512): the sample
// loop of models/fatchord_version.py:201-241 for up to 16 rows per XCD (128 per launch), e.g. the
// folds of fold_with_overlap (:293-340; BASELINE config 2 batched: 10 folds, config 3: 115 folds)
// or independent utterances.
//
// The weights of the loop are held once per XCD, spread over its 32 CUs as MFMA A operands:
// workgroup c (4 waves, one per SIMD) owns GRU units 16c..16c+15 (both GRUs) and fc rows
// 16c..16c+15; wave w multiplies the K window [128w, 128w + 128) of every one of the eleven 16-row
// weight sets (fatchord_xcdm.h, MSet): 11 × 32 floats per lane, eight sets in the 256 AGPRs (the
// MFMAs are inline asm with "a" operands, hazards handled by hand) and W_hh1 in VGPRs.  ≤ 2 quads
// of 4 batch rows: v_mfma_f32_4x4x1_16b_f32 — 16 blocks of (4 weight rows × 1 k) · (1 k × 4 batch
// rows) per instruction, block b = 4s' + g takes row group g and k-slice s' of the window; 3–4
// quads: v_mfma_f32_16x16x4_f32 (16 batch rows on N, K reduced inside).  The activations (B
// operands) of the window come from the packed hop vectors: each wave polls only its own
// 128-wide slice of every vector, stages it in LDS (XOR-swizzled) and reads it back as B.  The
// partial sums of the four k-slices and four waves are left unreduced in LDS; the threads that
// finish each layer (one unit or fc row and batch row each) sum them in a fixed order.
//
// Per step t (x = x_{t-1} of every row):
//   A  GRU1 of the own units (gate math; W_hh1·h1_{t-1} from the previous step)  → publish h1  [hop H1]
//   B  h1 slice → W_ih2·h1 (3 sets)                                              → barrier
//   C  GRU2 gate math → h2, y = x_I + h1 + h2                                     → publish y, h2 [hop Y]
//   D  W_hh1·h1 from the staged h1 slice (the next step's GRU1; fills hop Y's window)
//   E  y slice → fc1 (1 set)                                                      → barrier
//   F  fc1 epilogue (relu, V1 = fc1's a3 part + bias)                             → publish f1  [hop F1]
//   G  h2 slice → W_hh2·h2 (the next step's GRU2; fills hop F1's window)
//   H  f1 slice → fc2 (1 set)                                                     → barrier
//   I  fc2 epilogue → f2 → barrier → fc3 partial logits of the 16 own f2 rows      → publish     [hop F2]
//   J  sample (utils/distribution.py:87-123): ≤ 4 rows per XCD — every workgroup sums all 32
//      producers' partials of every row and samples it itself (waves 0..3, one row each);
//      more rows — workgroup c samples row c alone and publishes x [hop X], every workgroup
//      gathers the x of all rows (a fifth hop instead of 32× the partial-logit traffic)
// The conditioning terms of step t + 1 (terms GEMM, capi.cpp) and its sampler noise are loaded
// by waves 4..7 after their f1 poll and stored into an LDS ring before the step's last barrier.
//
// Membership as in fatchord_xcd.hip (XCC id + per-XCD arrival counter; bounded waits).  fp32,
// sums re-associated (MoL tolerance-checked against the oracle like the other kernels).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fatchord_loop.h"
#include "fatchord_xcd.h"
#include "fatchord_xcdm.h"
#include "mfma_device.h"
#include "wrnn_device.h"
#include "xcd_device.h"

namespace wrnn {

// fc3 partials wave-local (no barrier) from this many quads per XCD on: at B = 115 (4 quads)
// 12.97 → 12.87 µs/step; at 1 quad (B ≤ 32) the barrier form is faster (5.29 vs 5.35 at B = 10,
// 6.00 vs 6.12 at B = 32), at 2 quads neutral (profiles/r04_ab_xcdm_fc3_local.log)
#ifndef WRNN_XCDM_PART_BATCH
#define WRNN_XCDM_PART_BATCH 1   // GRU2 epilogue: operands hoisted above the barrier, the three gate partials' loads issued together (0: A/B)
#endif
#ifndef WRNN_XCDM_FC3_LOCAL_MINQ
#define WRNN_XCDM_FC3_LOCAL_MINQ 3
#endif

// Σ of the wave's four k-slices (lanes l, l ^ 16, l ^ 32, l ^ 48): identical bits in all four
__device__ __forceinline__ f4v kslice_sum(f4v d) {
    return f4v{cross_rows(d.x), cross_rows(d.y), cross_rows(d.z), cross_rows(d.w)};
}

// Σ of the four waves' partials of one output, fixed order
__device__ __forceinline__ float sum8(const float *p) {
    static_assert(kMWaves == 4, "one float4 of wave partials per output");
    const f4v u = lds4(p);
    return (u.x + u.y) + (u.z + u.w);
}

// A packed hop vector (fatchord_xcdm.h): the slot of step t, and its publish (a plain 4-byte
// store that stays in the XCD's L2, as xpub)
// (slot index made wave-uniform explicitly: otherwise the step-parity select is taken as
// divergent and every poll's buffer descriptor sits in a waterfall loop)
__device__ __forceinline__ float *pvec(unsigned long long *xg, int hop, int t) {
    const int slot = __builtin_amdgcn_readfirstlane(2 * (hop - MH_H1) + (t & 1));
    return reinterpret_cast<float *>(xg + kMPackOff) + (size_t)slot * kMVec;
}
// (a NaN whose bits equal kMEmpty — a NaN input can carry that payload through the layers — is
// published as the canonical quiet NaN, so a real value never reads as "empty")
__device__ __forceinline__ void ppub(float *p, float v) {
    const unsigned u = __float_as_uint(v);
    __hip_atomic_store(reinterpret_cast<unsigned *>(p), u == kMEmpty ? 0x7FC00000u : u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void pclear(float *p) {
    __hip_atomic_store(reinterpret_cast<unsigned *>(p), kMEmpty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// all four floats of a polled float4 published (none still empty)
__device__ __forceinline__ bool pfull(u4v v) {
    return (v.x != kMEmpty) & (v.y != kMEmpty) & (v.z != kMEmpty) & (v.w != kMEmpty);
}

// Poll wave w's slice [kMK·w, kMK·w + kMK) of a packed hop vector for every quad: lane l reads
// the float4s (row 4q + 2h + (l >> 5), columns kMK·w + 4(l & 31) + {0..3}), h = 0, 1.  Bounded.
template <int NQ>
__device__ __forceinline__ void mpoll(const float *vec, int w, int *ctl, long long timeout, int step, int hop,
                                      int *lds_abort, int lane, u4v (&v)[kMPP * NQ]) {
    const __amdgpu_buffer_rsrc_t r = hop_rsrc(reinterpret_cast<const unsigned long long *>(vec));
    const int off = kMK * w * 4 + mpoll_lane_off(lane);
    const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (;;) {
#pragma unroll
        for (int i = 0; i < kMPP * NQ; ++i) v[i] = ld16_sc1(r, off + mpoll_row(i) * 512 * 4);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < kMPP * NQ; ++i) ok &= pfull(v[i]);
        if (__ballot(!ok) == 0) return;   // wave-uniform exit
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

// polled float4s → the wave's staging area ([quad][row j4][64], XOR-swizzled by 4·j4)
// (quads q0 .. q0 + NQ - 1 of the wave's staging image; the 16x16x4 form's swizzle depends on
// the absolute row; a float4 of 4 columns stays contiguous under both swizzles)
template <int NQ, bool kBig>
__device__ __forceinline__ void mstage(float *stg, int q0, int lane, const u4v (&v)[kMPP * NQ]) {
#pragma unroll
    for (int i = 0; i < kMPP * NQ; ++i) {
        const int q = q0 + i / kMPP, j4 = mpoll_row(i) - 4 * (i / kMPP) + lane / (kMK / 4), kk = mpoll_col(lane);
        const int at = kBig ? mstg16_at(4 * q + j4, kk) : q * kMStg + mstg_at(j4, kk);
        *reinterpret_cast<u4v *>(stg + at) = v[i];
    }
}

// Poll + stage a wave's slice of all NQ quads, at most four quads (8 float4s) per poll round
template <int NQ, int Q0 = 0>
__device__ __forceinline__ void mgather(const float *vec, float *stg, int w, int *ctl, long long timeout, int step,
                                        int hop, int *lds_abort, int lane) {
    if constexpr (Q0 < NQ) {
        constexpr int G = NQ - Q0 < 4 ? NQ - Q0 : 4;
        u4v v[kMPP * G];
        mpoll<G>(vec + (size_t)Q0 * 4 * 512, w, ctl, timeout, step, hop, lds_abort, lane, v);
        mstage<G, xcdm_big(NQ)>(stg, Q0, lane, v);
        mgather<NQ, Q0 + G>(vec, stg, w, ctl, timeout, step, hop, lds_abort, lane);
    }
}

// A poll of the first G quads of a wave's slice that rides along an off-critical MFMA layer: the
// layer calls step(jc) at the start of each of its 8 k-chunks, and the poll's loads are issued
// once, at chunk kAt, so that the rest of the layer's MFMAs cover their round trip; finish()
// checks them after the layer (a wait only if they have not landed) and falls back to the
// bounded blocking poll (mpoll) if some element was still empty.  (Checking inside the
// layer would stall it: reading the loaded registers waits for the loads, landed or not.)
struct MPollNone {
    __device__ __forceinline__ void step(int) {}
};
template <int G, int kAt>
struct MPoll {
    u4v v[G > 0 ? kMPP * G : 1];
    __amdgpu_buffer_rsrc_t r;
    int off;
    __device__ __forceinline__ MPoll(const float *vec, int w, int lane) : off(0) {
        if constexpr (G > 0) {
            r = hop_rsrc(reinterpret_cast<const unsigned long long *>(vec));
            off = kMK * w * 4 + mpoll_lane_off(lane);
        }
    }
    __device__ __forceinline__ void step(int jc) {
        if constexpr (G > 0) {
            if (jc == kAt) {
#pragma unroll
                for (int i = 0; i < kMPP * G; ++i) v[i] = ld16_sc1(r, off + mpoll_row(i) * 512 * 4);
            }
        }
    }
    __device__ __forceinline__ void finish(const float *vec, int w, int *ctl, long long timeout, int step_, int hop,
                                           int *lds_abort, int lane) {
        if constexpr (G > 0) {
            // the loaded registers pass through an empty volatile asm here, so the check (and its
            // s_waitcnt) cannot be hoisted into the layer's MFMA stream (volatile asm, kept in
            // order): hipcc otherwise tests each float4 right after its load and stalls the layer
#pragma unroll
            for (int i = 0; i < kMPP * G; ++i) asm volatile("" : "+v"(v[i]));
            bool ok = true;
#pragma unroll
            for (int i = 0; i < kMPP * G; ++i) ok &= pfull(v[i]);
            if (__ballot(!ok) != 0) mpoll<G>(vec, w, ctl, timeout, step_, hop, lds_abort, lane, v);
        }
    }
};

// the wave's partials of every (row of the set, batch row of quad q), k-slices unreduced: lane
// l = 16·sp + 4g + j holds rows 4g + i (i = 0..3) of batch row 4q + j over k-slice sp →
// P[set][wave][row][n][sp] (row stride xcdm_pstride_row: the 64 lanes of one store hit 64 banks)
template <int NQ, int NS, int NC>
__device__ __forceinline__ void mput(f4v (&acc)[NS][NC], float *P, int q, int lane, int wave) {
    constexpr int S = xcdm_pstride_row(NQ);
    const int g = (lane >> 2) & 3, n = 4 * q + (lane & 3), sp = lane >> 4;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        f4v d = acc[s][0];
#pragma unroll
        for (int cc = 1; cc < NC; ++cc) d += acc[s][cc];
        float *p = P + ((s * kMWaves + wave) * 16 + 4 * g) * S + 4 * n + sp;
        p[0] = d.x;
        p[S] = d.y;
        p[2 * S] = d.z;
        p[3 * S] = d.w;
    }
}

// Σ over waves (and k-slices) of the partials of output (set·16 + row) i, batch row n; fixed order
template <int NQ>
__device__ __forceinline__ float mpart(const float *P, int i, int n) {
    if constexpr (xcdm_big(NQ)) {
        return sum8(P + (i * (4 * NQ) + n) * kMWaves);
    } else {
        constexpr int S = xcdm_pstride_row(NQ);
        const int s = i >> 4, r = i & 15;
        f4v u[kMWaves];
#pragma unroll
        for (int w = 0; w < kMWaves; ++w) u[w] = lds4(P + ((s * kMWaves + w) * 16 + r) * S + 4 * n);
        float t[kMWaves];
#pragma unroll
        for (int w = 0; w < kMWaves; ++w) t[w] = (u[w].x + u[w].y) + (u[w].z + u[w].w);
        return (t[0] + t[1]) + (t[2] + t[3]);
    }
}

// mpart of rows i0, i0 + 16, i0 + 32 (the r, z, n gate rows of a unit) with every load issued
// before the first add (a scheduling barrier between: hipcc pairs loads with their adds, one LDS
// round trip per pair)
template <int NQ>
__device__ __forceinline__ void mpart3(const float *P, int i0, int n, float (&out)[3]) {
    if constexpr (xcdm_big(NQ)) {
        static_assert(kMWaves == 4, "one float4 of wave partials per output");
        f4v u[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) u[q] = lds4(P + ((i0 + 16 * q) * (4 * NQ) + n) * kMWaves);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 3; ++q) out[q] = (u[q].x + u[q].y) + (u[q].z + u[q].w);
    } else {
        constexpr int S = xcdm_pstride_row(NQ);
        f4v u[3][kMWaves];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int i = i0 + 16 * q, ss = i >> 4, r = i & 15;
#pragma unroll
            for (int w = 0; w < kMWaves; ++w) u[q][w] = lds4(P + ((ss * kMWaves + w) * 16 + r) * S + 4 * n);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            float t[kMWaves];
#pragma unroll
            for (int w = 0; w < kMWaves; ++w) t[w] = (u[q][w].x + u[q][w].y) + (u[q][w].z + u[q][w].w);
            out[q] = (t[0] + t[1]) + (t[2] + t[3]);
        }
    }
}

// One layer: NS sets from S0 against every quad of the staged slice, the wave's partials to P.
// MFMA order: k-chunk (4 columns) outer, then column, quad, set; NC accumulator chains per
// (quad, set) (column j → chain j % NC).  A dependent v_mfma_f32_4x4x1_16b_f32 with srcC = the
// previous dst costs no stall from three interleaved chains up (tools/xcdm_layer_bench.hip), and
// one-set layers measured no faster with 3 or 4 chains than with 2.
// kLdsA (RAW fc3, NS = 1): the set's A operands come from LDS ([kMJ / 4][64 lanes][4], AL = the
// wave's image), read a k-chunk ahead like B.
template <int NQ, int S0, int NS, int NC, typename Hook = MPollNone, bool kLdsA = false>
__device__ __forceinline__ void mlayer(const float (&A)[kMSets][kMJ], const float *stg, float *P, int lane, int wave,
                                       Hook &&hook = Hook{}, const float *AL = nullptr) {
    constexpr bool kAgpr = !kLdsA && S0 < MS_HH1;
    const int j4 = lane & 3, sp = lane >> 4;
    f4v acc[NQ][NS][NC];
    f4v al[2];
    if constexpr (kLdsA) al[0] = lds4(AL + lane * 4);
    // B operands double-buffered: chunk jc + 1's LDS reads are in flight during chunk jc's MFMAs
    // (the asm MFMAs are volatile, so hipcc would not hoist a read above them by itself)
    f4v b[2][NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) b[0][q] = lds4(stg + q * kMStg + mstg_at(j4, kMJ * sp));
#pragma unroll
    for (int jc = 0; jc < kMJ / 4; ++jc) {
        hook.step(jc);
        if (jc + 1 < kMJ / 4) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) b[(jc + 1) & 1][q] = lds4(stg + q * kMStg + mstg_at(j4, kMJ * sp + 4 * (jc + 1)));
            if constexpr (kLdsA) al[(jc + 1) & 1] = lds4(AL + ((jc + 1) * 64 + lane) * 4);
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * jc + jj;
#pragma unroll
            for (int q = 0; q < NQ; ++q)
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    float av;
                    if constexpr (kLdsA) av = al[jc & 1][jj];
                    else av = A[S0 + s][j];
                    if (j < NC) mfma_first<kAgpr>(acc[q][s][j % NC], av, b[jc & 1][q][jj]);
                    else mfma_acc<kAgpr>(acc[q][s][j % NC], av, b[jc & 1][q][jj]);
                }
        }
    }
    mfma_drain_begin();
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) mfma_tie(acc[q][s][cc]);
#pragma unroll
    for (int q = 0; q < NQ; ++q) mput<NQ, NS, NC>(acc[q], P, q, lane, wave);
}

// The same layer with v_mfma_f32_16x16x4_f32 (≥ 3 quads): lane l = 16g + n takes batch row n and
// columns kMK·w + kMJ·g + i of MFMA i (the A operands are the 4x4x1 form's, lane for lane: row
// l & 15, column kMK·w + kMJ·(l >> 4) + i); the K reduction happens inside the MFMA, so lane l
// ends with rows 4(l >> 4) + r, r = 0..3, of batch row n, summed over the wave's whole window.
template <int NQ, int S0, int NS, int NC, typename Hook = MPollNone, bool kLdsA = false>
__device__ __forceinline__ void mlayer16(const float (&A)[kMSets][kMJ], const float *stg, float *P, int lane, int wave,
                                         Hook &&hook = Hook{}, const float *AL = nullptr) {
    constexpr bool kAgpr = !kLdsA && S0 < MS_HH1;
    constexpr int NR = 4 * NQ;
    const int n = lane & 15, g = lane >> 4;
    f4v acc[NS][NC];
    f4v b[2], al[2];
    b[0] = lds4(stg + mstg16_at(n, kMJ * g));
    if constexpr (kLdsA) al[0] = lds4(AL + lane * 4);
#pragma unroll
    for (int ic = 0; ic < kMJ / 4; ++ic) {
        hook.step(ic);
        if (ic + 1 < kMJ / 4) {
            b[(ic + 1) & 1] = lds4(stg + mstg16_at(n, kMJ * g + 4 * (ic + 1)));
            if constexpr (kLdsA) al[(ic + 1) & 1] = lds4(AL + ((ic + 1) * 64 + lane) * 4);
        }
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            const int i = 4 * ic + ii;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                float av;
                if constexpr (kLdsA) av = al[ic & 1][ii];
                else av = A[S0 + s][i];
                if (i < NC) mfma16_first<kAgpr>(acc[s][i % NC], av, b[ic & 1][ii]);
                else mfma16_acc<kAgpr>(acc[s][i % NC], av, b[ic & 1][ii]);
            }
        }
    }
    mfma16_drain_begin();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) mfma_tie(acc[s][cc]);
    if (n < NR) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            f4v d = acc[s][0];
#pragma unroll
            for (int cc = 1; cc < NC; ++cc) d += acc[s][cc];
            float *p = P + ((s * 16 + 4 * g) * NR + n) * kMWaves + wave;
            p[0] = d.x;
            p[NR * kMWaves] = d.y;
            p[2 * NR * kMWaves] = d.z;
            p[3 * NR * kMWaves] = d.w;
        }
    }
}


// accumulator chains per (quad, set): back-to-back accumulation into one chain costs nothing
// extra from three independent chains up (tools/xcdm_layer_bench.hip)
template <int NQ, int NS>
struct MChains {
    static constexpr int v = NQ * NS >= 3 ? 1 : 2;
};

// the layer in the kernel's MFMA form (optionally with a poll riding along)
template <int NQ, int S0, int NS, typename Hook = MPollNone>
__device__ __forceinline__ void mlayer_any(const float (&A)[kMSets][kMJ], const float *stg, float *P, int lane, int wave,
                                           Hook &&hook = Hook{}) {
    // (16x16x4: ≥ 3 sets interleaved already cover its ≈ 40-cycle dependent latency)
    // (one set: four chains, so the ≈ 40-cycle dependent latency never stalls the 32-cycle issue)
    if constexpr (xcdm_big(NQ)) mlayer16<NQ, S0, NS, NS == 1 ? 4 : 2>(A, stg, P, lane, wave, hook);
    else mlayer<NQ, S0, NS, MChains<NQ, NS>::v>(A, stg, P, lane, wave, hook);
}
// one set whose A operands are in LDS (RAW fc3); partials in the set-0 slot of P
template <int NQ>
__device__ __forceinline__ void mlayer_lds(const float (&A)[kMSets][kMJ], const float *AL, const float *stg, float *P,
                                           int lane, int wave) {
    if constexpr (xcdm_big(NQ)) mlayer16<NQ, 0, 1, 2, MPollNone, true>(A, stg, P, lane, wave, MPollNone{}, AL);
    else mlayer<NQ, 0, 1, MChains<NQ, 1>::v, MPollNone, true>(A, stg, P, lane, wave, MPollNone{}, AL);
}

// quads polled beside an off-critical layer (all of them: ≤ 8 float4s per lane, the registers
// the tagged form's two quads took), and the k-chunk at which its loads are issued
#ifndef WRNN_XCDM_F1_ALL
#define WRNN_XCDM_F1_ALL 1
#endif
#ifndef WRNN_XCDM_RIDE_AT
#define WRNN_XCDM_RIDE_AT 3
#endif
template <int NQ>
struct MRide {
    static constexpr int G = NQ;
    static constexpr int at = WRNN_XCDM_RIDE_AT;
};

// Poll + stage the hop vector `vec` (all quads) with its first MRide group already polled by `pr`
template <int NQ>
__device__ __forceinline__ void mgather_rest(MPoll<MRide<NQ>::G, MRide<NQ>::at> &pr, const float *vec,
                                             float *stg, int w, int *ctl, long long timeout, int step, int hop,
                                             int *lds_abort, int lane) {
    constexpr int G = MRide<NQ>::G;
    if constexpr (G > 0) {
        pr.finish(vec, w, ctl, timeout, step, hop, lds_abort, lane);
        mstage<G, xcdm_big(NQ)>(stg, 0, lane, pr.v);
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mgather<NQ, G>(vec, stg, w, ctl, timeout, step, hop, lds_abort, lane);
}

// MoL sample of XCD row n by one wave: Σ of the 32 producers' partial logits + b3, then
// mol_sample_pairs (xcd_device.h) with the row's noise terms (ring).  Wave-uniform result.
__device__ __forceinline__ float msample(const unsigned long long *f2, int n, uint32_t tag, const float *nz,
                                         const float *cst, int *ctl, long long timeout, int step, int *lds_abort,
                                         int lane) {
    const int jp = lane & 15, pg = lane >> 4;
    const float ua = nz[jp < 5 ? 2 * jp : 0], ub = nz[jp < 5 ? 2 * jp + 1 : 0], u10 = nz[10];
    const float b3a = cst[MC_B3 + 2 * jp], b3b = cst[MC_B3 + 2 * jp + 1];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const __amdgpu_buffer_rsrc_t rf = hop_rsrc(f2);
    const int goff = ((n * kXcdWgs + 8 * pg) * 32 + 2 * jp) * 8;
    const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    u4v v[8];
    for (;;) {   // one wave-uniform exit; the values taken after the loop
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = ld16_sc1(rf, goff + m * 32 * 8);
        bool ok = true;
#pragma unroll
        for (int m = 0; m < 8; ++m) ok &= (v[m].y == tag) & (v[m].w == tag);
        if (__ballot(!ok) == 0) break;
        if ((++spins & 63u) == 0) {
            const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > timeout;
            const bool other = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (late || other) {
                if (late) record_abort(ctl, -4, step, MH_F2, blockIdx.x);
                *lds_abort = 1;
                break;
            }
        }
    }
    float pa[8], pb[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        pa[m] = __uint_as_float(v[m].x);
        pb[m] = __uint_as_float(v[m].z);
    }
#pragma unroll
    for (int w = 4; w >= 1; w /= 2)
#pragma unroll
        for (int m = 0; m < w; ++m) {
            pa[m] += pa[m + w];
            pb[m] += pb[m + w];
        }
    cross_rows_pair(pa[0], pb[0]);
    const float la = pa[0] + b3a, lb = pb[0] + b3b;   // logits 2jp, 2jp+1
    return mol_sample_pairs(la, lb, ua, ub, u10, jp);
}

// RAW sample of XCD row n by one wave (fatchord_version.py:231-237): the row's 512 logits (32
// producers × 16 own classes, published as granules n·512 + class) polled as pairs — lane l holds
// classes 2(l + 64i) + {0, 1}, i < 4 — then softmax → Categorical renormalisation → argmax(p / q)
// with the row's Exp(1) draws q (the fp32 operations of wrnn_device.h:raw_sample; first index on
// ties).  Returns the label, wave-uniform.
__device__ __forceinline__ int rsample(const unsigned long long *lg, int n, uint32_t tag, const f2v (&q)[4], int *ctl,
                                       long long timeout, int step, int *lds_abort, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const __amdgpu_buffer_rsrc_t rf = hop_rsrc(lg);
    const int goff = (n * kMRawNC + 2 * lane) * 8;
    const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    u4v v[4];
    bool dead = false;
    for (;;) {   // one wave-uniform exit; the values taken after the loop
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ld16_sc1(rf, goff + i * 128 * 8);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 4; ++i) ok &= (v[i].y == tag) & (v[i].w == tag);
        if (__ballot(!ok) == 0) break;
        if ((++spins & 63u) == 0) {
            const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > timeout;
            const bool other = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (late || other) {
                if (late) record_abort(ctl, -4, step, MH_LG, blockIdx.x);
                *lds_abort = 1;
                dead = true;
                break;
            }
        }
    }
    if (dead) return 0;
    float e[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        e[2 * i] = __uint_as_float(v[i].x);
        e[2 * i + 1] = __uint_as_float(v[i].z);
    }
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, e[k]);
    m = wave_max(m);
    float s1 = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        e[k] = expf(e[k] - m);
        s1 += e[k];
    }
    s1 = wave_sum(s1);
    float s2 = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        e[k] = e[k] / s1;
        s2 += e[k];
    }
    s2 = wave_sum(s2);
    float bv = -INFINITY;
    int bi = 0x7FFFFFFF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        am_merge(bv, bi, (e[2 * i] / s2) / q[i].x, 2 * (lane + 64 * i));
        am_merge(bv, bi, (e[2 * i + 1] / s2) / q[i].y, 2 * (lane + 64 * i) + 1);
    }
    return WRNN_XCD_ORDERED_ARGMAX ? wave_argmax_fast(bv, bi) : wave_argmax(bv, bi);
}

// diagnostics (template kDbg, WRNN_DEBUG_STAMPS=1): lane 0 of every wave stamps the shader clock
// at the phase boundaries below into LDS for kMDbgSteps steps from t0 + kMDbgSkip (global stores
// would sit in vmcnt ahead of the polls); copied out after the loop; tools/stamps_xcdm.py reads them
#define MST(kk)                                                                                              \
    do {                                                                                                     \
        if (kDbg && lane == 0 && (unsigned)(t - a.t0 - kMDbgSkip) < (unsigned)kMDbgSteps)                   \
            dbgs[((t - a.t0 - kMDbgSkip) * kMWaves + wave) * kMStamps + (kk)] =                              \
                (unsigned)__builtin_amdgcn_s_memtime();                                                      \
    } while (0)

// kRaw: the RAW (9-bit softmax) head — f2 published as a hop vector, fc3 (own 16 classes, A
// operands in LDS) on the gathered f2 slice, the logits a sixth hop, rsample instead of msample;
// the Exp(1) draws always come from `noise` (Philox pre-filled by the host).
template <int NQ, bool kDbg, bool kRaw>
__global__ __launch_bounds__(kMThreads, 1) void fatchord_xcdm_kernel(XcdmArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int NR = 4 * NQ;
    constexpr bool kTwoLevel = NQ >= 2;
    // fc3 partials by the waves that own the rows, no barrier (WRNN_XCDM_FC3_LOCAL_MINQ: from how
    // many quads on; measured in profiles/r04_ab_xcdm_fc3_local.log)
    constexpr bool kFc3Local = NQ >= WRNN_XCDM_FC3_LOCAL_MINQ;
    constexpr int N = kXcdWgs * kMRing;   // the compact terms record (capi.cpp: d_xmWt)
    const XcdmLds ll = xcdm_lds_layout(NQ, kDbg, kRaw);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int kStgQ = xcdm_big(NQ) ? kMQuadMax : NQ;   // staged quads per wave
    float *stg_h1 = smem + ll.stg_h1 + wave * kStgQ * kMStg, *stg = smem + ll.stg + wave * kStgQ * kMStg;
    float *pbig = smem + ll.pbig, *phh1 = smem + ll.phh1, *pfc1 = smem + ll.pfc1, *pfc2 = smem + ll.pfc2;
    float *gh1 = smem + ll.gh1, *gh2 = smem + ll.gh2, *f2s = smem + ll.f2, *ring = smem + ll.ring, *nzr = smem + ll.nz;
    float *cst = smem + ll.cst, *w3s = smem + ll.w3, *xs = smem + ll.xs, *a3s = smem + ll.a3;
    int *misc = reinterpret_cast<int *>(smem + ll.misc);
    int *abort_flag = misc;
    unsigned *dbgs = reinterpret_cast<unsigned *>(smem + ll.dbg);

    // ---- membership: XCD k (launch rows k, k + 8, ...) and index c within it
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
    const int RX = (a.nb - k + kXcds - 1) / kXcds;     // rows n < RX of this XCD: launch row k + 8n
    const int t_end = a.t0 + a.Lc;
    unsigned long long *xg = a.xg + (size_t)k * kMXcdStride;
    const float *S = a.slab + (size_t)c * a.s.total;
    // the terms record of (step t, row n): ring float4 f of this workgroup at + mterm_off(c, 4f)
    auto TERMS = [&](int t, int n) { return a.terms + ((size_t)(t - a.t0) * a.nb + (k + kXcds * n)) * N; };

    // ---- register-resident MFMA A operands: the wave's K window of all eleven sets
    float A[kMSets][kMJ];
#pragma unroll
    for (int s = 0; s < kMSets; ++s)
#pragma unroll
        for (int j = 0; j < kMJ; ++j) A[s][j] = S[a.s.a + ((wave * kMSets + s) * kMJ + j) * 64 + lane];

    // roles: (unit / fc row u, batch row n) for the layer epilogues; (logit j, row n) for fc3
    // (16·NR = 64·NQ threads = waves 0..NQ-1: tested on the SGPR wave index, so the epilogue role
    // branches are scalar instead of exec-mask branches)
    static_assert(16 * NR == 64 * NQ, "epilogue threads are whole waves");
    const bool gru = wave < NQ;
    // the off-critical recurrent sums (Σ W_hh·h of the next step; 16 partials each in the 4x4x1
    // form) are taken by the waves that do not sample, while the samplers run J: waves ≥ aux_w0
    // (none when every wave samples: then the epilogue threads take them in F and I)
    const int aux_w0 = xcdm_big(NQ) ? kMWaves : kTwoLevel ? 1 : RX;
    const int gu = tid & 15, gn = tid >> 4;
    constexpr int kRingF4 = kMRing / 4;   // float4s of one row's terms
    // ring loader threads: all (≤ 4 rows per XCD: sampler waves store their loads after sampling,
    // the others before it) or waves 1..3 (two-level sampler: they store before it, wave 0 samples)
    constexpr int kLdThreads = kTwoLevel ? kMThreads - 64 : kMThreads;
    constexpr int kRingLd = (NR * kRingF4 + kLdThreads - 1) / kLdThreads;   // ring loads per thread

    // terms of step t → ring slot t & 1 (rows n < RX; the rest stay zero)
    auto ring_at = [&](int t) { return ring + (t & 1) * NR * kMRing; };
    auto nz_at = [&](int t) { return nzr + (t & 1) * NR * kMNoise; };
    auto noise_uu = [&](int t, int n, int kk) -> float {
        const int lr = k + kXcds * n;
        if (a.noise) return a.noise[((size_t)(t - a.nz_t0) * a.nz_ts + a.nz_b0 + lr) * 11 + kk];
        // opaque seed: hipcc would otherwise hoist all ten Philox round keys out of the step loop
        // into (spilled) VGPRs
        unsigned long long seed = a.seed;
        asm volatile("" : "+s"(seed));
        return philox_noise(seed, (unsigned long long)(a.row0 + lr), (uint32_t)t, (uint32_t)kk, 1);
    };

    // ---- prologue: constants, zeroed accumulators / ring, state, the terms of step t0
    for (int i = tid; i < kMCst; i += kMThreads) cst[i] = S[a.s.cst + i];
    if constexpr (kRaw) {
        for (int i = tid; i < kMWaves * kMJ * 64; i += kMThreads) a3s[i] = S[a.s.a3 + i];
    } else {
        for (int i = tid; i < 32 * kMW3Stride; i += kMThreads) w3s[i] = S[a.s.w3 + i];
        for (int i = tid; i < 2 * NR * kMNoise; i += kMThreads) nzr[i] = 0.0f;
    }
    for (int i = tid; i < 2 * NR * kMRing; i += kMThreads) ring[i] = 0.0f;
    for (int i = tid; i < 3 * 16 * NR; i += kMThreads) gh1[i] = gh2[i] = 0.0f;
    if (tid < 16) xs[tid] = 0.0f;
    __syncthreads();
    const bool resume = a.t0 > 0;
    float *st = a.state + ((size_t)k * kXcdWgs + c) * kMStateW;
    float h1v = 0.0f, h2v = 0.0f;   // h1 / h2 of (unit gu, row gn): this thread's recurrent state
    if (resume) {
        if (gru) {
            h1v = st[gu * 16 + gn];
            h2v = st[256 + gu * 16 + gn];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                gh1[(q * 16 + gu) * NR + gn] = st[512 + (q * 16 + gu) * 16 + gn];
                gh2[(q * 16 + gu) * NR + gn] = st[1280 + (q * 16 + gu) * 16 + gn];
            }
        }
        if (tid < RX) xs[tid] = st[2048 + tid];
    }
    for (int i = tid; i < RX * kRingF4; i += kMThreads) {
        const int n = i / kRingF4, f = i - n * kRingF4;
        *reinterpret_cast<f4v *>(ring_at(a.t0) + n * kMRing + 4 * f) =
            *reinterpret_cast<const f4v *>(TERMS(a.t0, n) + mterm_off(c, 4 * f));
    }
    if constexpr (!kRaw)
        for (int i = tid; i < 11 * RX; i += kMThreads) {
            const int n = i / 11, kk = i - 11 * n;
            nz_at(a.t0)[n * kMNoise + kk] = mol_noise_term(noise_uu(a.t0, n, kk), kk);
        }
    __syncthreads();

    for (int t = a.t0; t < t_end; ++t) {
        // per-thread indices re-derived every step from an opaque copy of threadIdx.x: otherwise
        // hipcc hoists every per-thread address out of the loop and keeps them all live in VGPRs,
        // which the weights leave no room for (spills)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, gu = tid & 15, gn = tid >> 4;
        const uint32_t tag = (uint32_t)t + 1u;
        const float *rg = ring_at(t);
        const bool more = t + 1 < t_end;
        float x = 0.0f;
        MST(0);
        if (kDbg && lane == 0 && (unsigned)(t - a.t0 - kMDbgSkip) < (unsigned)kMDbgSteps)
            dbgs[((t - a.t0 - kMDbgSkip) * kMWaves + wave) * kMStamps + kMStamps - 1] = (unsigned)__builtin_amdgcn_s_memrealtime();
        // ---- A: GRU1 (:208-210) of unit gu, row gn: W_ih1·x_I is rank-1 in x given the terms
        if (gru) {
            x = xs[gn];
            const float *tr = rg + gn * kMRing;
            float sr, sz, gin, ghn;
            {
                const int i0 = gu, i1 = 16 + gu, i2 = 32 + gu;
                sr = (gh1[i0 * NR + gn] + cst[MC_BHH1 + i0]) + (tr[MT_P1 + gu * 3 + 0] + cst[MC_BIH1 + i0]);
                sz = (gh1[i1 * NR + gn] + cst[MC_BHH1 + i1]) + (tr[MT_P1 + gu * 3 + 1] + cst[MC_BIH1 + i1]);
                gin = tr[MT_P1 + gu * 3 + 2] + cst[MC_BIH1 + i2];
                ghn = gh1[i2 * NR + gn] + cst[MC_BHH1 + i2];
            }
            const float r = sigmoid_(fmaf(x, cst[MC_Q1 + gu], sr));
            const float z = sigmoid_(fmaf(x, cst[MC_Q1 + 16 + gu], sz));
            const float nn = tanh_(fmaf(x, cst[MC_Q1 + 32 + gu], gin) + ghn * r);
            h1v = (h1v - nn) * z + nn;
            ppub(pvec(xg, MH_H1, t) + gn * 512 + 16 * c + gu, h1v);
        }
        MST(1);
        // ---- B: the h1 slice → W_ih2[:, :R]·h1 (the GRU2 input gates, :213-214)
        {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            mgather<NQ>(pvec(xg, MH_H1, t), stg_h1, wave, a.ctl, a.timeout_ticks, t, MH_H1, abort_flag, lane);
            MST(2);
            // every workgroup's h1_t is here, so every consumer has read all of step t - 1: empty
            // this thread's elements of the other slot (step t + 1's), ordered before the y publish
            if (gru) {
                const int e = gn * 512 + 16 * c + gu;
#pragma unroll
                for (int hv = MH_H1; hv < (kRaw ? MH_F2 + 1 : MH_F2); ++hv) pclear(pvec(xg, hv, t + 1) + e);
            }
            mlayer_any<NQ, MS_IH2, 3>(A, stg_h1, pbig, lane, wave);
            MST(3);
        }
        // C's operands that the layer does not produce, read above the barrier (in registers
        // across it: only the partials' loads remain after it)
        // (not for the 4-quad RAW head: 4 more VGPRs than it has)
        constexpr bool kHoistC = WRNN_XCDM_PART_BATCH && !(kRaw && NQ == 4);
        float c_pi[3], c_gh[3], c_xi = 0.0f;
        if (kHoistC && gru) {
            const float *tr = rg + gn * kMRing;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int i = q * 16 + gu;
                c_pi[q] = fmaf(x, cst[MC_Q2 + i], tr[MT_P2 + gu * 3 + q]) + cst[MC_BIH2 + i];
                c_gh[q] = gh2[i * NR + gn] + cst[MC_BHH2 + i];
            }
            c_xi = fmaf(cst[MC_WI0 + gu], x, tr[MT_CI + gu]);
            asm volatile("" : "+v"(c_pi[0]), "+v"(c_pi[1]), "+v"(c_pi[2]), "+v"(c_gh[0]), "+v"(c_gh[1]), "+v"(c_gh[2]),
                         "+v"(c_xi));
        }
        bar();
        MST(4);
        // ---- C: GRU2 (:212-214) gate math → h2; y = (x_I + h1) + h2 (:212, :216)
        if (gru) {
            const float *tr = rg + gn * kMRing;
            float gi[3], gh[3], xi;
            if constexpr (kHoistC) {
                float pp[3];
                mpart3<NQ>(pbig, gu, gn, pp);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    gi[q] = pp[q] + c_pi[q];
                    gh[q] = c_gh[q];
                }
                xi = c_xi;
            } else {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int i = q * 16 + gu;
                    gi[q] = mpart<NQ>(pbig, i, gn) + (fmaf(x, cst[MC_Q2 + i], tr[MT_P2 + gu * 3 + q]) + cst[MC_BIH2 + i]);
                    gh[q] = gh2[i * NR + gn] + cst[MC_BHH2 + i];
                }
                xi = fmaf(cst[MC_WI0 + gu], x, tr[MT_CI + gu]);
            }
            h2v = gru_gate_math(gi[0], gi[1], gi[2], gh[0], gh[1], gh[2], h2v);
            const float y = (xi + h1v) + h2v;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the slot clears of B first
            ppub(pvec(xg, MH_Y, t) + gn * 512 + 16 * c + gu, y);
            ppub(pvec(xg, MH_H2, t) + gn * 512 + 16 * c + gu, h2v);
        }
        MST(5);
        // ---- D: W_hh1·h1 (the GRU1 terms of step t + 1; carried to the next chunk after the
        // last one) from the staged h1 slice, with the y poll of E riding along (hop Y's window)
        MPoll<MRide<NQ>::G, MRide<NQ>::at> py(pvec(xg, MH_Y, t), wave, lane);
        mlayer_any<NQ, MS_HH1, 3>(A, stg_h1, phh1, lane, wave, py);
        MST(6);
        // ---- E: the y slice → fc1 (:217-218)
        {
            mgather_rest<NQ>(py, pvec(xg, MH_Y, t), stg, wave, a.ctl, a.timeout_ticks, t, MH_Y, abort_flag, lane);
            MST(7);
        }
        // h2 was published with y: its poll rides along fc1 and is checked in G, after F
        MPoll<MRide<NQ>::G, MRide<NQ>::at> ph(pvec(xg, MH_H2, t), wave, lane);
        mlayer_any<NQ, MS_FC1, 1>(A, stg, pfc1, lane, wave, ph);
        MST(8);
        bar();
        MST(9);
        // ---- F: fc1 epilogue → f1; Σ W_hh1·h1 for the next GRU1
        // The f1 store is issued by EVERY thread (WRNN_XCDM_F1_ALL): threads past the epilogue
        // roles (rows ≥ NR, unused rows of the 16-row vector storage, never polled) store 0.  With
        // the store only on the epilogue path, hipcc's wait-count merge at the join made the h2
        // check below (its loads issued in fc1, before this store) wait vmcnt(0) — i.e. for this
        // store's acknowledgement too — on the path that has the store; with one store on every
        // path it waits vmcnt(1), for the loads alone.
        if (WRNN_XCDM_F1_ALL) {
            float f1v = 0.0f;
            if (gru) {
                const float f = mpart<NQ>(pfc1, gu, gn) + rg[gn * kMRing + MT_V1 + gu];
                f1v = f > 0.0f ? f : 0.0f;
            }
            ppub(pvec(xg, MH_F1, t) + gn * 512 + 16 * c + gu, f1v);
        }
        if (gru) {
            if (!WRNN_XCDM_F1_ALL) {
                const float f = mpart<NQ>(pfc1, gu, gn) + rg[gn * kMRing + MT_V1 + gu];
                ppub(pvec(xg, MH_F1, t) + gn * 512 + 16 * c + gu, f > 0.0f ? f : 0.0f);
            }
            if (aux_w0 >= kMWaves) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int i = q * 16 + gu;
                    gh1[i * NR + gn] = mpart<NQ>(phh1, i, gn);
                }
            }
        }
        MST(10);
        // ---- G: the h2 slice → W_hh2·h2 (the next step's GRU2), with the f1 poll of H riding
        // along (hop F1's window); f1 is staged once the layer's B reads of the h2 slice are done
        {
            mgather_rest<NQ>(ph, pvec(xg, MH_H2, t), stg, wave, a.ctl, a.timeout_ticks, t, MH_H2, abort_flag, lane);
            MST(11);
            MPoll<MRide<NQ>::G, MRide<NQ>::at> pf(pvec(xg, MH_F1, t), wave, lane);
            mlayer_any<NQ, MS_HH2, 3>(A, stg, pbig, lane, wave, pf);
            MST(12);
            // ---- H: the f1 slice → fc2 (:220-221)
            mgather_rest<NQ>(pf, pvec(xg, MH_F1, t), stg, wave, a.ctl, a.timeout_ticks, t, MH_F1, abort_flag, lane);
            MST(13);
            mlayer_any<NQ, MS_FC2, 1>(A, stg, pfc2, lane, wave);
            MST(14);
        }
        bar();
        MST(15);
        // the terms and noise of step t + 1 → registers now, into the ring before the last barrier
        // (issued here, they have landed by the sampler's poll of hop F2)
        f4v rl[kRingLd];
        float uu = 0.0f;
        // (direct sampler: loader index counted from the last thread, so that with few rows the
        // loads sit in waves that do not sample and store them before J)
        const int lt = kTwoLevel ? tid - 64 : kMThreads - 1 - tid;
        if (more && lt >= 0) {
            // through a buffer descriptor on step t + 1's record (uniform) + a 32-bit offset, the
            // segment offset by selects: the pointer form compiled to divergent branches and 64-bit
            // address math, ≈ 50 instructions per load — it held the loader waves' fc2 epilogue
            // (and with it the fc3 partials hop F2 waits for) ≈ 1 000 cycles behind wave 0's
            const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<float *>(a.terms + (size_t)(t + 1 - a.t0) * a.nb * N), 0, 0x7fffffff, 0x00020000);
#pragma unroll
            for (int i = 0; i < kRingLd; ++i) {
                const int idx = lt + kLdThreads * i;
                if (idx < RX * kRingF4) {
                    const int n = idx / kRingF4, s4 = 4 * (idx - n * kRingF4);
                    if constexpr (kRaw && NQ == 4) {   // (the RAW 4-quad head has no VGPRs to spare: as before)
                        rl[i] = *reinterpret_cast<const f4v *>(TERMS(t + 1, n) + mterm_off(c, s4));
                    } else {
                        int off = kMG0 + c * 64 + s4;
                        off = s4 >= MT_P2 ? kMG1 + c * 48 + (s4 - MT_P2) : off;
                        off = s4 >= MT_V1 ? kMG2 + c * 32 + (s4 - MT_V1) : off;   // = mterm_off(c, s4)
                        rl[i] = __builtin_bit_cast(
                            f4v, __builtin_amdgcn_raw_buffer_load_b128(trs, ((k + kXcds * n) * N + off) * 4, 0, 0));
                    }
                }
            }
            if (!kRaw && lt < 11 * RX) {
                const int n = lt / 11, kk = lt - 11 * n;
                uu = noise_uu(t + 1, n, kk);
            }
        }
        // RAW: the Exp(1) draws of the row this wave samples (step t), pairs of classes
        // 2(lane + 64i) + {0, 1} — issued here, landed by the logits poll
        f2v qv[4];
        const int sn = kTwoLevel ? c : wave;                          // sampled row
        const bool smp = kTwoLevel ? (wave == 0 && c < RX) : (wave < RX);
        if constexpr (kRaw) {
            if (smp) {
                const float *qr = a.noise + ((size_t)(t - a.nz_t0) * a.nz_ts + a.nz_b0 + k + kXcds * sn) * kMRawNC;
#pragma unroll
                for (int i = 0; i < 4; ++i) qv[i] = *reinterpret_cast<const f2v *>(qr + 2 * (lane + 64 * i));
            }
        }
        auto ring_store = [&]() {
            if (more && lt >= 0) {
                float *rn = ring_at(t + 1);
#pragma unroll
                for (int i = 0; i < kRingLd; ++i) {
                    const int idx = lt + kLdThreads * i;
                    if (idx < RX * kRingF4) {
                        const int n = idx / kRingF4, f = idx - n * kRingF4;
                        *reinterpret_cast<f4v *>(rn + n * kMRing + 4 * f) = rl[i];
                    }
                }
                if (!kRaw && lt < 11 * RX) {
                    const int n = lt / 11, kk = lt - 11 * n;
                    nz_at(t + 1)[n * kMNoise + kk] = mol_noise_term(uu, kk);
                }
            }
        };
        // ---- I: fc2 epilogue → f2 (LDS); Σ W_hh2·h2 for the next GRU2
        if (gru) {
            const float f = mpart<NQ>(pfc2, gu, gn) + rg[gn * kMRing + MT_V2 + gu];
            if constexpr (kRaw) ppub(pvec(xg, MH_F2, t) + gn * 512 + 16 * c + gu, f > 0.0f ? f : 0.0f);
            else f2s[gn * kMW3Stride + gu] = f > 0.0f ? f : 0.0f;
            if (aux_w0 >= kMWaves) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int i = q * 16 + gu;
                    gh2[i * NR + gn] = mpart<NQ>(pbig, i, gn);
                }
            }
        }
        MST(16);
        if constexpr (kRaw) {
            // fc3 (:223) rows of the own 16 classes on the gathered f2 slice → logits [hop LG]
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            mgather<NQ>(pvec(xg, MH_F2, t), stg, wave, a.ctl, a.timeout_ticks, t, MH_F2, abort_flag, lane);
            MST(17);
            mlayer_lds<NQ>(A, a3s + wave * kMJ * 64, stg, pfc1, lane, wave);
            bar();
            if (gru) xpub(xg + kMHopOff[MH_LG] + gn * 512 + 16 * c + gu, tag, mpart<NQ>(pfc1, gu, gn) + cst[MC_B3 + gu]);
        } else if (kFc3Local) {
            // fc3 (:223) partial logits of the own 16 f2 rows, by the wave that wrote those rows' f2
            // (gru threads: row gn = tid >> 4, whole waves): a wave-local LDS round trip instead of
            // a workgroup barrier; lane l: logits (l & 15) and (l & 15) + 16 of row 4·wave + (l >> 4)
            if (gru) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                const int fn = 4 * wave + (lane >> 4);
                f4v fv[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) fv[q] = lds4(f2s + fn * kMW3Stride + 4 * q);
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int fj = (lane & 15) + 16 * hh;
                    f4v wv[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) wv[q] = lds4(w3s + fj * kMW3Stride + 4 * q);
                    float p = 0.0f;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        p = fmaf(wv[q].x, fv[q].x, p);
                        p = fmaf(wv[q].y, fv[q].y, p);
                        p = fmaf(wv[q].z, fv[q].z, p);
                        p = fmaf(wv[q].w, fv[q].w, p);
                    }
                    xpub(xg + kMHopOff[MH_F2] + (fn * kXcdWgs + c) * 32 + fj, tag, p);
                }
            }
            MST(17);
        } else {
            bar();
            MST(17);
            // fc3 (:223) partial logits of the own 16 f2 rows: logit fj of row fn
#pragma unroll
            for (int i = tid; i < 32 * NR; i += kMThreads) {
                const int fj = i & 31, fn = i >> 5;
                f4v wv[4], fv[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    wv[q] = lds4(w3s + fj * kMW3Stride + 4 * q);
                    fv[q] = lds4(f2s + fn * kMW3Stride + 4 * q);
                }
                float p = 0.0f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    p = fmaf(wv[q].x, fv[q].x, p);
                    p = fmaf(wv[q].y, fv[q].y, p);
                    p = fmaf(wv[q].z, fv[q].z, p);
                    p = fmaf(wv[q].w, fv[q].w, p);
                }
                xpub(xg + kMHopOff[MH_F2] + (fn * kXcdWgs + c) * 32 + fj, tag, p);
            }
        }
        MST(18);
        if (kTwoLevel || wave >= RX) ring_store();
        if (wave >= aux_w0) {
            const int na = (kMWaves - aux_w0) * 64;
            for (int e = tid - aux_w0 * 64; e < 3 * 16 * NR; e += na) {
                const int i = e / NR, n = e - i * NR;
                gh1[e] = mpart<NQ>(phh1, i, n);
                gh2[e] = mpart<NQ>(pbig, i, n);
            }
        }
        MST(19);
        // ---- J: sample (:225-229; RAW :231-237) row n of this XCD, wave-uniform x
        const float *nz = nz_at(t);
        auto sample_row = [&](int n) -> float {
            if constexpr (kRaw) {
                const int lab = rsample(xg + kMHopOff[MH_LG], n, tag, qv, a.ctl, a.timeout_ticks, t, abort_flag, lane);
                if (lane == 0 && a.labels && (kTwoLevel || c == 0))
                    a.labels[(size_t)(a.b0 + k + kXcds * n) * a.L + t] = lab;
                return label_to_x(lab, kMRawNC);
            } else {
                return msample(xg + kMHopOff[MH_F2], n, tag, nz + n * kMNoise, cst, a.ctl, a.timeout_ticks, t, abort_flag,
                               lane);
            }
        };
        if (!kTwoLevel) {
            if (wave < RX) {
                const float xn = sample_row(wave);
                if (lane == 0) {
                    xs[wave] = xn;
                    if (c == 0) a.out[(size_t)(a.b0 + k + kXcds * wave) * a.L + t] = xn;
                }
            }
        } else if (wave == 0) {
            if (c < RX) {   // this workgroup samples row c and publishes its x
                const float xn = sample_row(c);
                if (lane == 0) {
                    xpub(xg + kMHopOff[MH_X] + c, tag, xn);
                    a.out[(size_t)(a.b0 + k + kXcds * c) * a.L + t] = xn;
                }
            }
            // every workgroup: the x of all rows (lane n < RX polls row n)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned long long *gx = xg + kMHopOff[MH_X] + (lane < RX ? lane : 0);
            const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
            unsigned spins = 0;
            unsigned long long g;
            for (;;) {
                g = __hip_atomic_load(gx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool ok = lane >= RX || (uint32_t)(g >> 32) == tag;
                if (__ballot(!ok) == 0) break;
                if ((++spins & 63u) == 0) {
                    const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                    const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    if (late || other) {
                        if (late) record_abort(a.ctl, -4, t, MH_X, blockIdx.x);
                        *abort_flag = 1;
                        break;
                    }
                }
            }
            if (lane < RX) xs[lane] = __uint_as_float((uint32_t)g);
        }
        MST(20);
        // ring: the terms and noise of step t + 1 (loaded in H)
        if (!kTwoLevel && wave < RX) ring_store();
        MST(21);
        bar();
        if (*abort_flag) return;
    }
    if (kDbg && a.dbg) {
        __syncthreads();
        for (int i = tid; i < kMDbgSteps * kMWaves * kMStamps; i += kMThreads) {
            const int stp = i / (kMWaves * kMStamps), w = (i / kMStamps) % kMWaves, kk = i % kMStamps;
            a.dbg[(((size_t)blockIdx.x * kMWaves + w) * kMDbgSteps + stp) * kMStamps + kk] = dbgs[i];
        }
    }
    // ---- carry the recurrent state to the next time chunk
    if (gru) {
        st[gu * 16 + gn] = h1v;
        st[256 + gu * 16 + gn] = h2v;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            st[512 + (q * 16 + gu) * 16 + gn] = gh1[(q * 16 + gu) * NR + gn];
            st[1280 + (q * 16 + gu) * 16 + gn] = gh2[(q * 16 + gu) * NR + gn];
        }
    }
    if (tid < RX) st[2048 + tid] = xs[tid];
}

// The in-kernel Philox draws of launch rows [0, nb) for steps [t0, t0 + Lc) into the injected-noise
// layout [Lc][nb][K] (philox_noise keyed by (seed, row0 + row, step, k) exactly as the loop
// kernels key them: bit-identical audio), so the loop only loads them.  K = 11, mol = 1: the MoL
// uniforms; K = 2Q, mol = 0: the deepmind Exp(1) draws.
__global__ void philox_fill_kernel(float *out, unsigned long long seed, long long row0, int nb, int t0, int Lc, int K,
                                   int mol) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)Lc * nb * K) return;
    const int kk = (int)(i % K), lr = (int)((i / K) % nb), dt = (int)(i / ((long long)K * nb));
    out[i] = philox_noise(seed, (unsigned long long)(row0 + lr), (uint32_t)(t0 + dt), (uint32_t)kk, mol);
}

hipError_t launch_philox_fill(float *out, unsigned long long seed, long long row0, int nb, int t0, int Lc, int K, int mol,
                              hipStream_t st) {
    const long long n = (long long)Lc * nb * K;
    hipLaunchKernelGGL(philox_fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, seed, row0, nb, t0, Lc,
                       K, mol);
    return hipGetLastError();
}

// RAW kernels have no stamp variant (the stamp buffer does not fit LDS beside the fc3 operands)
static const void *xcdm_kernel(int nq, bool dbg, bool raw) {
    static const void *k[3][kMQuadMax] = {
        {(const void *)fatchord_xcdm_kernel<1, false, false>, (const void *)fatchord_xcdm_kernel<2, false, false>,
         (const void *)fatchord_xcdm_kernel<3, false, false>, (const void *)fatchord_xcdm_kernel<4, false, false>},
        {(const void *)fatchord_xcdm_kernel<1, true, false>, (const void *)fatchord_xcdm_kernel<2, true, false>,
         (const void *)fatchord_xcdm_kernel<3, true, false>, (const void *)fatchord_xcdm_kernel<4, true, false>},
        {(const void *)fatchord_xcdm_kernel<1, false, true>, (const void *)fatchord_xcdm_kernel<2, false, true>,
         (const void *)fatchord_xcdm_kernel<3, false, true>, (const void *)fatchord_xcdm_kernel<4, false, true>}};
    return k[raw ? 2 : dbg ? 1 : 0][nq < 1 ? 0 : nq > kMQuadMax ? kMQuadMax - 1 : nq - 1];
}

hipError_t launch_xcdm(const XcdmArgs &a, int nq, bool raw, hipStream_t st) {
    XcdmArgs args = a;
    void *params[] = {&args};
    const bool dbg = !raw && a.dbg != nullptr;
    const void *kf = xcdm_kernel(nq, dbg, raw);
    return hipLaunchKernel(kf, dim3(kXcds * kXcdWgs), dim3(kMThreads), params,
                           xcdm_lds_layout(nq, dbg, raw).total * sizeof(float), st);
}

hipError_t prepare_xcdm_kernel(int max_lds_bytes) {
    for (int v = 0; v < 3; ++v)
        for (int nq = 1; nq <= kMQuadMax; ++nq) {
            hipError_t e = hipFuncSetAttribute(xcdm_kernel(nq, v == 1, v == 2), hipFuncAttributeMaxDynamicSharedMemorySize,
                                               max_lds_bytes);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

// largest quad count whose launch is co-resident (one workgroup per CU); 0 if none
hipError_t xcdm_max_quads(int max_lds_bytes, bool raw, int *nq_max) {
    *nq_max = 0;
    for (int nq = 1; nq <= kMQuadMax; ++nq) {
        if (xcdm_lds_layout(nq, !raw, raw).total * sizeof(float) > (size_t)max_lds_bytes) break;
        int n = 0;
        for (int dbg = 0; dbg < (raw ? 1 : 2); ++dbg) {
            const size_t lds = xcdm_lds_layout(nq, dbg, raw).total * sizeof(float);
            hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xcdm_kernel(nq, dbg, raw), kMThreads, lds);
            if (e != hipSuccess) return e;
            if (n < 1) return hipSuccess;
        }
        *nq_max = nq;
    }
    return hipSuccess;
}

}  // namespace wrnn
