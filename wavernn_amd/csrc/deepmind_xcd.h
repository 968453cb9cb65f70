// Shared between the host launcher (capi.cpp) and deepmind_xcd.hip: the XCD-resident kernel of the
// dual coarse/fine softmax WaveRNN (models/deepmind_version.py:75-165) — up to 4 rows
// (utterances) on each XCD, 32 per launch, all stepping through one copy of the weights held in
// the XCD's 32 CUs as fp32 MFMA A operands (v_mfma_f32_4x4x1_16b_f32: the 4 rows of an XCD are the
// MFMA's batch columns), every hand-off kept in the XCD's L2.
//
// Shapes: hidden 896 (split 448), quantisation 256 — BASELINE config 5.
#pragma once
#include <stdint.h>

#include "fatchord_xcd.h"

namespace wrnn {

constexpr int kDxH = 896, kDxS = 448, kDxQ = 256;
constexpr int kDxWaves = 4, kDxThreads = 64 * kDxWaves;
constexpr int kDxRowsXcd = 4;                    // rows per XCD (one batch quad)
constexpr int kDxRowsMax = kXcds * kDxRowsXcd;   // rows per launch
constexpr int kDxU = kDxS / kXcdWgs;             // 14 coarse + 14 fine units per workgroup
constexpr int kDxUO2 = kDxQ / kXcdWgs;           // 8 rows of O2 / O4 per workgroup
constexpr int kDxKW = kDxS / kDxWaves;           // 112: K window of a wave in each half of h

// Workgroup c of an XCD owns coarse units 14c + u and fine units S + 14c + u (u < 14): their 84
// rows of R (WG-local row (half·3 + g)·14 + u, g = u/r/e gate; R row g·H + half·S + 14c + u,
// deepmind_version.py:116-119), rows 14c..14c+13 of O1 / O3 and 8c..8c+7 of O2 / O4.  Wave w
// multiplies the columns [112w, 112w + 112) of each half of h (coarse, fine) — of o1 / o3 for
// O2 / O4 — so that each half's MFMAs can run as soon as that half has been gathered.
//
// MFMA A operands per lane (slab [kDxWaves][kDxA][64 lanes]), lane l = 4b + j (block b):
//   R sets 0..4 (WG rows 16s..16s+15; 4 row groups × 4 k-slices: g = b & 3, s' = b >> 2):
//       DA_R + 56s + m:   R[row 16s + 4g + j][col(m)], m < 28: 112w + 28s' + m; else S + 112w + 28s' + m - 28
//   R quarter set (WG rows 80..83 = fine e-gate units 10..13; 1 row group × 16 k-slices s' = b):
//       DA_RQ + m:        R[row 80 + j][112w + 7s' + m] (m < 7), S + 112w + 7s' + m - 7 (m ≥ 7)
//   O1 / O3 (rows 14c + 4g + j, rows ≥ 14 zero; 4 × 4 as R): DA_O1 / DA_O3 + m: [col 112w + 28s' + m]
//   O2 / O4 (rows 8c + 4g + j; 2 row groups × 8 k-slices: g = b & 1, s' = b >> 1):
//       DA_O2 / DA_O4 + m:  [col 112w + 14s' + m], m < 14
enum DxA { DA_R = 0, DA_O1 = 280, DA_O3 = 308, DA_RQ = 336, DA_O2 = 350, DA_O4 = 364, kDxA = 378 };

// Per-workgroup constants (LDS)
enum DxCst {
    DC_B1 = 0,        // O1 bias of rows 14c + r (16, zero padded)
    DC_B3 = 16,       // O3 bias
    DC_B2 = 32,       // O2 bias of rows 8c + r
    DC_B4 = 40,       // O4 bias
    DC_IC = 48,       // I_coarse rows (g·S + 14c + u): [3][14][2]
    DC_IF = 132,      // I_fine rows: [3][14][3]
    DC_BU = 258,      // bias_u / bias_r / bias_e of the own units: [2 halves][14]
    DC_BR = 286,
    DC_BE = 314,
    kDxCst = 344,
};

struct DxSlab {
    int a;       // [kDxWaves][kDxA][64]
    int cst;     // [kDxCst]
    int total;   // floats per workgroup
};
__host__ __device__ inline DxSlab dx_slab_layout() {
    DxSlab s;
    s.a = 0;
    s.cst = kDxWaves * kDxA * 64;
    s.total = s.cst + kDxCst;
    return s;
}

// Hand-off vectors of one XCD, row n (0..3) = launch row k + 8n; granules {tag = step + 1, value}
enum DxHop { DX_HC = 0, DX_O1 = 1, DX_LC = 2, DX_HF = 3, DX_O3 = 4, DX_LF = 5, kDxHops = 6 };
#ifndef WRNN_DX_PAD
#define WRNN_DX_PAD 1   // 448-wide hop rows padded to 16 granules per workgroup (one 128-B line each)
#endif
// row stride (granules) of the 448-wide hop vectors (h_c, o1, h_f, o3): with WRNN_DX_PAD each
// workgroup's 14 granules start a 128-byte line of their own (16 granules, the last two written
// as pads with the tag) instead of sharing lines with the neighbouring workgroups
constexpr int kDxSP = WRNN_DX_PAD ? 16 * kXcdWgs : kDxS;
constexpr int kDxUP = kDxSP / kXcdWgs;   // granules per workgroup and row (16 or 14)
constexpr long long kDxHopOff[kDxHops] = {0, 4 * kDxSP, 8 * kDxSP, 8 * kDxSP + 4 * kDxQ, 12 * kDxSP + 4 * kDxQ,
                                          16 * kDxSP + 4 * kDxQ};
constexpr long long kDxXcdStride = 16 * kDxSP + 8 * kDxQ + 64;   // granules per XCD

// Carried state per workgroup (time-chunked launches): h of the own units [4 rows][28], the R·h
// partials (LDS image of ll.pr / ll.prq), previous labels [2][4]
constexpr int kDxPR = 5 * kDxWaves * 16 * 20;       // R sets: [set][wave][row 16][n 4 + 1 pad][4 k-slices]
constexpr int kDxPRQ = kDxWaves * 4 * 4 * 16;       // R quarter set: [wave][row 4][n 4][16 k-slices]
constexpr int kDxStateW = 4 * 2 * kDxU + kDxPR + kDxPRQ + 8;

constexpr int kDxDbgSteps = 32, kDxDbgSkip = 16, kDxStamps = 26;

struct DxArgs {
    const float *slab;               // [256 workgroups][DxSlab.total]
    const float *noise;              // [.][nz_ts][2Q] q_coarse | q_fine, Exp(1) draws
    long long nz_ts;                 // rows per noise step (the caller's Bt or the Philox chunk's nb)
    int nz_t0, nz_b0;                // noise step / row of launch step t0 / launch row 0
    float *out;                      // [Bt][L] combined sample (utils/dsp.py:33) as float
    int32_t *labels;                 // [Bt][L] or nullptr
    float *state;                    // [8 XCDs][32][kDxStateW]
    unsigned long long *xg;          // [8][kDxXcdStride]
    int *members;                    // [8] arrival counters (zeroed per launch)
    int *ctl;
    long long timeout_ticks;
    int L, t0, Lc, Bt, b0, nb;       // nb ≤ 32 launch rows: b0 .. b0 + nb - 1
    DxSlab s;
    unsigned *dbg;                   // stamps (WRNN_DEBUG_STAMPS) or nullptr
};

struct DxLds {
    int stg, ao, pr, prq, rs, po1, po3, po2, po4, nz, cst, lab, misc, gbc, dbg, total;
};
constexpr int kDxST = kDxKW + 4;   // staged slice row stride (floats)
// A operands read from LDS instead of registers (the quarter set and O2 / O4: 42 per lane and
// wave): [wave][DA_RQ .. DA_O4 + 14)[64 lanes]
constexpr int kDxAL = kDxA - DA_RQ;   // 42
__host__ __device__ inline DxLds dx_lds_layout(bool dbg = false) {
    DxLds l;
    int o = 0;
    l.stg = o;  o += 3 * kDxWaves * 4 * kDxST;     // staged slices: [h_f | o1 then o3 | h_c][wave][n][kDxST]
    l.ao = o;   o += kDxWaves * kDxAL * 64;
    l.pr = o;   o += kDxPR;
    l.prq = o;  o += kDxPRQ;
    l.rs = o;   o += 84 * 4;                       // Σ R·h of the own 84 gate rows [rr][n]
    l.po1 = o;  o += kDxWaves * 16 * 20;
    l.po3 = o;  o += kDxWaves * 16 * 20;
    l.po2 = o;  o += kDxWaves * 8 * 4 * 8;         // [wave][row 8][n 4][8 k-slices]
    l.po4 = o;  o += kDxWaves * 8 * 4 * 8;
    l.nz = o;   o += 2 * 4 * 2 * kDxQ;             // log q of steps t, t + 1 (by parity) [2][n][2Q]
    l.cst = o;  o += kDxCst + 4;
    l.lab = o;  o += 16;                           // previous coarse [4], fine [4], c_t [4]
    l.misc = o; o += 8;                            // [0] abort flag, [1] member index
    l.gbc = o;  o += kDxWaves * 3 * 4 * 64;        // R·h group B after its coarse half: [wave][set 3, 4, quarter][4][64]
    l.dbg = o;  o += dbg ? kDxDbgSteps * kDxWaves * kDxStamps : 0;
    l.total = o;
    return l;
}

}  // namespace wrnn
