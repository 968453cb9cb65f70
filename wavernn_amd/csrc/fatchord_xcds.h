// Shared between the host launcher (capi.cpp) and fatchord_xcds.hip: the XCD-resident MoL
// kernel for rnn 896 with 4×4 block-sparse GRU matrices (BASELINE config 4, pruning.py) — one
// utterance (row) per XCD, its whole sample loop on that XCD's 32 CUs, every hand-off inside the
// XCD's L2 (the same scheme as fatchord_xcd.h for dense rnn 512).
#pragma once
#include <stdint.h>

#include "fatchord_xcd.h"

namespace wrnn {

constexpr int kSR = 896;             // rnn dims
constexpr int kSU = kSR / kXcdWgs;   // 28 GRU units per workgroup
constexpr int kSUB = kSU / 4;        // 7 four-unit block-rows per gate per workgroup
constexpr int kSBR = 3 * kSUB;       // 21 gate block-rows per matrix per workgroup (br = q·7 + ub)
constexpr int kSNB = 32;             // nonzero 4×4 blocks per block-row at most (2 per lane of a 16-lane engine)
constexpr int kSPairs = kSR / 128;   // 7: 16-byte granule pairs per lane to poll an rnn-wide vector

// Conditioning terms of one step for one workgroup (columns of the terms GEMM), floats:
//   [0,84) P1 = W_ih1·cI, [84,168) P2 = W_ih2·[cI; a2]   (index u·3 + gate, u = local unit)
//   [168,196) cI of the own units, [196,212) V1 = W1[:, R:]·a3 + b1, [212,228) V2 = W2[:, F:]·a4 + b2
enum SXTerm { SX_P1 = 0, SX_P2 = 84, SX_CI = 168, SX_V1 = 196, SX_V2 = 212, kSTerms = 228 };

// Small per-workgroup vectors (LDS-resident), offsets within the cst block: q2 = W_ih2[:, :R]·W_I[:, 0]
// and the biases of both GRUs (own units, u·3 + q), W_I[:, 0] of the own units, b3 (padded to 32)
enum SXCst { SC_Q2 = 0, SC_BIH1 = 84, SC_BHH1 = 168, SC_BIH2 = 252, SC_BHH2 = 336, SC_WI0 = 420, SC_B3 = 448, kSCst = 480 };

// Per-workgroup weight slab (floats; column-block indices stored as int bits):
struct XcdsSlab {
    int wih2b;   // [21 block-rows][32 blocks][16]   W_ih2[:, :R] nonzero 4×4 blocks, row-major, zero-padded
    int whh1b;   // [21][32][16]                     W_hh1
    int whh2b;   // [21][32][16]                     W_hh2
    int wih2c;   // [21][32] int                     column-block index of each block (0 for padding)
    int whh1c;   // [21][32] int
    int whh2c;   // [21][32] int
    int w1;      // [16][896]   fc1 rows 16c + r (y part)
    int w2;      // [16][512]   fc2 rows 16c + r (f1 part)
    int w3;      // [16][32]    W3[j][16c + r] (j ≥ 30: 0)
    int q1a;     // [3][896]    W_ih1·W_I[:, 0], gate-major (all units)
    int cst;     // [kSCst]
    int total;
};

// Per-workgroup state carried between time chunks (floats):
// [h1 896 | sg 3584 (terms of the next step) | gh2 84 | h2own 28 | x | pad]
constexpr int kSStateW = 896 + 3584 + 84 + 28 + 4;

struct XcdsArgs {
    const float *slab;            // [kXcdWgs][slab.total]
    const float *terms;           // [Lc + 1][nb][kXcdWgs·kSTerms], row (t - t0)·nb + k
    const float *noise;           // [L][Bt][11] or nullptr (Philox)
    float *out;                   // [Bt][L]
    float *state;                 // [nb][kXcdWgs][kSStateW]
    unsigned long long *xg;       // [nb][kXXcdStride] granules
    int *members;                 // [kXcds] arrival counters (zeroed before the launch)
    int *ctl;                     // [0] abort, [1] code, [2] step, [3] hop, [4] wg
    unsigned long long seed;
    long long row0;               // global row id of XCD 0's row (Philox key: row0 + k)
    long long timeout_ticks;
    int L, t0, Lc, Bt, b0, nb;
    XcdsSlab s;
    unsigned *dbg;                // [nb·32][dbg_steps][kStamps] or nullptr
    int dbg_steps;
};

struct XcdsLds {
    int h1, h2, sg, w3, f2x, ring, nz, gh2, cst, xs, misc, whh1b, whh1c, whh2b, whh2c, total;
};

__host__ __device__ inline XcdsLds xcds_lds_layout() {
    XcdsLds l;
    int o = 0;
    // the small per-step arrays first (offsets < 64 KiB: lane address + instruction immediate)
    l.h1 = o;    o += kSR;
    l.h2 = o;    o += kSR;
    l.sg = o;    o += 4 * kSR;                // GRU1 terms of all units for the coming step
    l.w3 = o;    o += kXFcRows * 32;          // fc3 columns of the own f2 rows (waves 0..3)
    l.f2x = o;   o += 3 * 64;                 // waves 1..3's fc3 partials, handed to wave 0: (value, tag) pairs
    l.ring = o;  o += kXRing * kSTerms;
    l.nz = o;    o += kXRing * kXNoise;
    l.gh2 = o;   o += 88;                     // W_hh2·h2 of the own units (u·3 + q) for the next step
    l.cst = o;   o += kSCst;
    l.xs = o;    o += 4;                      // x, by step parity
    l.misc = o;  o += 8;                      // [0] abort, [1] member, flags (step + 1): [2] h2 gathered,
                                              // [3], [6], [7] f2x of wave 1 / 2 / 3 ready, [4] y gathered,
                                              // [5] f1 gathered
    l.whh1b = o; o += kSBR * kSNB * 16;
    l.whh1c = o; o += kSBR * kSNB;
    l.whh2b = o; o += kSBR * kSNB * 16;
    l.whh2c = o; o += kSBR * kSNB;
    l.total = o;
    return l;
}

}  // namespace wrnn
