// Shared between the host launcher (capi.cpp) and fatchord_xcdm.hip: the XCD-resident MoL kernel
// for MANY rows — up to 16 rows (utterances or folds) on each XCD, all of them stepping together
// through one copy of the weights held in the XCD's 32 CUs, the matvecs on the matrix cores
// (v_mfma_f32_4x4x1_16b_f32 at ≤ 2 quads of 4 batch rows, v_mfma_f32_16x16x4_f32 at 3–4 quads),
// every hand-off kept in the XCD's L2.
//
// Shapes: rnn 512, fc 512, aux 32, MoL (30 classes) — BASELINE configs 2 (fold-batched) and 3 —
// or RAW 9-bit (512 classes, fatchord_version.py:231-237): fc3 is then a twelfth 16-row set (the
// own classes 16c..16c+15, A operands in LDS), f2 a full hop vector and the logits a sixth one.
#pragma once
#include <stdint.h>

#include "fatchord_xcd.h"

namespace wrnn {

// Four waves per workgroup, one per SIMD: the partial-sum epilogues (one float4 of wave partials
// per output, fatchord_xcdm.hip) and the K windows are written for exactly that.
constexpr int kMWaves = 4;                 // waves per workgroup (one per SIMD)
constexpr int kMThreads = 64 * kMWaves;
constexpr int kMQuadMax = 4;               // batch quads (4 rows) per XCD
constexpr int kMRowsXcd = 4 * kMQuadMax;   // rows per XCD
constexpr int kMRowsMax = kXcds * kMRowsXcd;   // rows per launch (128 ≥ config 3's 115 folds)
constexpr int kMK = 512 / kMWaves;         // K window of a wave: wave w multiplies columns [kMK·w, kMK·(w + 1))
constexpr int kMJ = kMK / 4;               // MFMAs per set and quad (4 k-slices of kMJ columns)
constexpr int kMPP = kMK / 64;             // 16-byte poll loads per lane and quad (4 rows × kMK packed floats)

// The eleven 16-row weight sets a workgroup c multiplies (rows of its units 16c..16c+15 / fc rows
// 16c..16c+15), register-resident as MFMA A operands (16 per set and wave: kMK / 4 k-slices)
enum MSet { MS_IH2 = 0, MS_FC1 = 3, MS_FC2 = 4, MS_HH2 = 5, MS_HH1 = 8, kMSets = 11 };
//   MS_IH2 + q: W_ih2[q·512 + 16c + u][:512]   MS_HH2 + q / MS_HH1 + q: W_hh2 / W_hh1 rows likewise
//   MS_FC1: fc1.weight[16c + r][:512]          MS_FC2: fc2.weight[16c + r][:512]
// A operand of set s, MFMA j (0..kMJ-1), lane l = 4b + j4 (block b = 4s' + g: row group g = b & 3,
// k-slice s' = b >> 2): W_s[row 4g + j4][kMK·w + kMJ·s' + j]  (slab [kMWaves][11][kMJ][64 lanes])

// Hand-off vectors of one XCD.  Row n (0..15) of the XCD = launch row k + 8n.
// Tagged granules {tag = step + 1, value}: F2 (MoL partial logits of producer c) at
// (n·32 + c)·32 + j, j < 32 (30, 31 zero); X (two-level sampler) at n; RAW: LG the logits
// (n·512 + class).
// Packed vectors (untagged fp32, two slots by step parity, kMPackOff granules in): H1 / Y / H2 /
// F1 (RAW: and the f2 vector, MH_F2) at slot·kMVec + n·512 + j (unit or fc row j).  An empty
// element holds kMEmpty (0xFFFFFFFF, a NaN pattern: ppub maps a published NaN of exactly these
// bits to the canonical 0x7FC00000, so no published value reads as empty); the producer of an
// element empties the other slot once its B poll of step t has seen every workgroup's h1_t —
// by then every consumer has read all of step t - 1 — and a later publish of its own orders the
// clear before step t + 1's polls.  Twice the values per 16-byte poll of the tagged form.
enum MHop { MH_H1 = 0, MH_Y = 1, MH_H2 = 2, MH_F1 = 3, MH_F2 = 4, MH_X = 5, MH_LG = 6, kMHops = 7 };
constexpr int kMPacked = 5;                // packed vectors: MH_H1 .. MH_F2
constexpr uint32_t kMEmpty = 0xFFFFFFFFu;
constexpr long long kMVec = (long long)kMRowsXcd * 512;
constexpr long long kMF2 = (long long)kMRowsXcd * kXcdWgs * 32;   // >= kMVec
constexpr long long kMHopOff[kMHops] = {0, kMVec, 2 * kMVec, 3 * kMVec, 4 * kMVec, 4 * kMVec + kMF2,
                                        4 * kMVec + kMF2 + 64};
constexpr long long kMPackOff = 5 * kMVec + kMF2 + 64;           // granules: the packed area
constexpr long long kMXcdStride = kMPackOff + kMPacked * kMVec;  // granules per XCD (packed: 2 floats each)
// (every word of the area starts as 0xFFFFFFFF: an empty packed element, a tag no step carries)
constexpr int kMRawNC = 512;        // RAW classes (bits = 9)
// MoL fc3 partials: the 16 fc3 columns of a logit and the 16 own f2 rows of a batch row are each
// read as four ds_read_b128; rows padded to 20 floats so the 16 lanes of a b128 phase hit distinct banks
constexpr int kMW3Stride = 20;

// Per-workgroup constants (LDS), gate-major: index q·16 + u
enum MCst { MC_Q1 = 0, MC_Q2 = 48, MC_BIH1 = 96, MC_BHH1 = 144, MC_BIH2 = 192, MC_BHH2 = 240, MC_WI0 = 288,
            MC_B3 = 304, kMCst = 336 };
//   q1 / q2: W_ih1 / W_ih2[:, :R] · W_I[:, 0] (the x column of the I layer folded into the gates),
//   biases of both GRUs, W_I[:, 0] of the own units, b3 (padded to 32; RAW: of the own classes)

struct XcdmSlab {
    int a;       // [kMWaves][kMSets][16][64]   MFMA A operands
    int a3;      // RAW: [kMWaves][kMJ / 4][64][4] fc3 A operands (own classes), copied to LDS
    int w3;      // [32][kMW3Stride]             W3[j][16c + r] at j·20 + r (j >= 30: 0)
    int cst;     // [kMCst]
    int total;
};

// Terms of one step for one row: P1 (48), cI (16), P2 (48), V1 (16), V2 (16) — the 144 of the XCD
// kernels' 160-slot record this kernel uses (compact weights d_xmWt: 32 × 144 rows)
constexpr int kMRing = 144;
// The terms GEMM is split into three groups so that each reads only the input columns it
// depends on (capi.cpp, generate_xcdm: 53 % of the FLOPs of one full-depth GEMM): [P1 | cI] on
// mel‖a1‖1, P2 on mel‖a1‖1‖a2, [V1 | V2] on a3‖a4‖1.  The record of one row-step is segmented by
// group, workgroup-major inside each — [(P1 ‖ cI) of wg 0..31 | P2 of wg 0..31 | (V1 ‖ V2) of
// wg 0..31] — so each group is one plain GEMM writing a contiguous row range, and a workgroup
// reads three runs of a row-step's record (256 B, 192 B, 128 B; measured against one 576-B run
// per workgroup and five runs segmented by type, profiles/r04_ab_terms_gemm.log).  The LDS ring
// keeps the workgroup's terms in run order (MT_ slots): float4 f of the runs is ring float4 f.
enum MTerm { MT_P1 = 0, MT_CI = 48, MT_P2 = 64, MT_V1 = 112, MT_V2 = 128 };
constexpr int kMG0 = 0, kMG1 = 32 * 64, kMG2 = kMG1 + 32 * 48, kMGEnd = kMG2 + 32 * 32;   // group offsets
static_assert(kMGEnd == kXcdWgs * kMRing, "segmented terms record");
// record offset of ring slot s (MT_ order) of workgroup c
__host__ __device__ inline int mterm_off(int c, int s) {
    return s < MT_P2 ? kMG0 + c * 64 + s : s < MT_V1 ? kMG1 + c * 48 + (s - MT_P2) : kMG2 + c * 32 + (s - MT_V1);
}
// the XT_ slot (XCD kernels' terms-GEMM weight rows, pack_xcd_terms_weights) of ring slot s
__host__ __device__ inline int mterm_xt(int s) {
    return s < MT_CI ? XT_P1 + s : s < MT_P2 ? XT_CI + (s - MT_CI) : s < MT_V1 ? XT_P2 + (s - MT_P2) : s;
}
constexpr int kMNoise = 12;                // 11 MoL sampler terms per row and step, padded

// Per-workgroup state carried between time chunks: h1 / h2 of the own units [16][16 rows],
// W_hh1·h1 / W_hh2·h2 [3][16][16], x [16]
constexpr int kMStateW = 256 + 256 + 768 + 768 + 16;

struct XcdmArgs {
    const float *slab;            // [kXcdWgs][slab.total]
    const float *terms;           // [Lc][nb][kXcdWgs·kMRing], row (t - t0)·nb + launch row
    const float *noise;           // uniforms of step t, launch row lr: noise[((t - nz_t0)·nz_ts + nz_b0 + lr)·11 + k],
                                  // or nullptr (in-kernel Philox)
    long long nz_ts;
    int nz_t0, nz_b0;
    float *out;                   // [Bt][L]
    int32_t *labels;              // RAW: [Bt][L] class labels, or nullptr
    float *state;                 // [kXcds][kXcdWgs][kMStateW]
    unsigned long long *xg;       // [kXcds][kMXcdStride] granules
    int *members;                 // [kXcds] arrival counters (zeroed before the launch)
    int *ctl;                     // [0] abort, [1] code, [2] step, [3] hop, [4] wg
    unsigned long long seed;
    long long row0;               // global row id of launch row 0 (Philox key: row0 + launch row)
    long long timeout_ticks;
    int L, t0, Lc, Bt, b0, nb;    // launch rows b0 .. b0 + nb - 1 of the call's Bt; nb <= kMRowsMax
    XcdmSlab s;
    unsigned *dbg;                // WRNN_DEBUG_STAMPS: [256 wg][kMWaves][kMDbgSteps][kMStamps] s_memtime, or nullptr
};
constexpr int kMStamps = 24, kMDbgSteps = 48, kMDbgSkip = 16;

struct XcdmLds {
    int stg_h1, stg, pbig, phh1, pfc1, pfc2, gh1, gh2, f2, ring, nz, cst, w3, a3, xs, misc, dbg, total;
};

// staging of a polled vector slice, per wave: [quad][4 rows][64], value k of row j4 at
// j4·64 + (k ^ 4·j4) (the XOR keeps the B-operand reads of the four rows on distinct banks)
constexpr int kMStg = 4 * kMK;
// lane l's float4 i (of kMPP·NQ) of a packed vector slice: quad i / kMPP; float4s
// p = l + 64·(i % kMPP) cover the 4 rows of the quad row-major (kMK / 4 per row)
__host__ __device__ constexpr int mpoll_row(int i) { return 4 * (i / kMPP) + (((i % kMPP) * 64) / (kMK / 4)); }
__host__ __device__ inline int mpoll_col(int lane) { return 4 * (lane % (kMK / 4)); }
__host__ __device__ inline int mpoll_lane_off(int lane) { return ((lane / (kMK / 4)) * 512 + mpoll_col(lane)) * 4; }
// staging position of (row j4, column kk): 4-float groups XOR-swizzled so that the B reads of the
// 16 (row, k-slice) combinations of a wave instruction fall on distinct bank groups
__host__ __device__ inline int mstg_at(int j4, int kk) {
    const int g = kk >> 2, sw = kMK == 128 ? (((g >> 4) & 1) << 2) | j4 : j4;
    return j4 * kMK + 4 * (g ^ sw) + (kk & 3);
}
// the 16x16x4 form (≥ 3 quads): all 16 rows of a wave's slice in one [16][kMK] image, row n's
// 4-float group g at g ^ n (the 16 rows of a B read fall on distinct bank groups)
__host__ __device__ inline int mstg16_at(int n, int kk) { return n * kMK + 4 * ((kk >> 2) ^ n) + (kk & 3); }
// quads whose MFMAs use v_mfma_f32_16x16x4_f32 (rows on N, no k-slices) instead of the 4x4x1 form
__host__ __device__ constexpr bool xcdm_big(int nq) { return nq >= 3; }

// floats of one set's cross-wave partials: [row][nr][wave] (16x16x4 form, k-slices reduced in
// the MFMA) or [wave][row][nr + 1 pad][4 k-slices] (4x4x1 form, k-slices left unreduced: the
// consumer sums 16 values instead of the producer running a permlane reduction)
__host__ __device__ constexpr int xcdm_pstride_row(int nq) { return 4 * (4 * nq) + 4; }
__host__ __device__ constexpr int xcdm_pset(int nq) {
    return xcdm_big(nq) ? 16 * 4 * nq * kMWaves : kMWaves * 16 * xcdm_pstride_row(nq);
}

__host__ __device__ inline XcdmLds xcdm_lds_layout(int nq, bool dbg = false, bool raw = false) {
    const int nr = 4 * nq, nq_stg = xcdm_big(nq) ? kMQuadMax : nq;
    XcdmLds l;
    int o = 0;
    l.stg_h1 = o; o += kMWaves * nq_stg * kMStg;   // the h1 slice (GRU2, then W_hh1)
    l.stg = o;    o += kMWaves * nq_stg * kMStg;   // y / h2 / f1 slices
    l.pbig = o;   o += 3 * xcdm_pset(nq);              // cross-wave partials: W_ih2·h1, then W_hh2·h2
    l.phh1 = o;   o += 3 * xcdm_pset(nq);              // W_hh1·h1
    l.pfc1 = o;   o += xcdm_pset(nq);
    l.pfc2 = o;   o += xcdm_pset(nq);
    l.gh1 = o;    o += 3 * 16 * nr;                    // Σ W_hh1·h1 (next step's GRU1)
    l.gh2 = o;    o += 3 * 16 * nr;                    // Σ W_hh2·h2 (next step's GRU2)
    l.f2 = o;     o += raw ? 0 : kMW3Stride * nr;      // MoL: f2 of the own rows (fc3 partials), [row][20]
    l.ring = o;   o += 2 * nr * kMRing;                // terms of steps t, t + 1 (by parity)
    l.nz = o;     o += raw ? 0 : 2 * nr * kMNoise;
    l.cst = o;    o += kMCst;
    l.w3 = o;     o += raw ? 0 : 32 * kMW3Stride;
    l.a3 = o;     o += raw ? kMWaves * kMJ * 64 : 0;   // RAW: fc3 A operands (LDS-resident)
    l.xs = o;     o += 16;
    l.misc = o;   o += 8;                              // [0] abort flag, [1] member index
    l.dbg = o;    o += dbg ? kMDbgSteps * kMWaves * kMStamps : 0;
    l.total = o;
    return l;
}

}  // namespace wrnn
