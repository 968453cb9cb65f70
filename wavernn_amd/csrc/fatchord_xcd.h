// Shared between the host launcher (capi.cpp) and fatchord_xcd.hip: the XCD-resident MoL
// kernel — one utterance (row) per XCD, its whole sample loop on that XCD's 32 CUs, every
// hand-off kept inside the XCD's L2.
#pragma once
#include <stdint.h>

namespace wrnn {

constexpr int kXcds = 8;            // XCDs of an MI355X (one row each)
constexpr int kXcdWgs = 32;         // workgroups (= CUs) per XCD, one per CU
constexpr int kXWaves = 8;          // compute waves per workgroup (two per SIMD), no loader wave
constexpr int kXThreads = 64 * kXWaves;
constexpr int kXUnits = 16;         // GRU units per workgroup (R / kXcdWgs), 2 per wave
constexpr int kXFcRows = 16;        // fc1 / fc2 rows per workgroup (F / kXcdWgs)
// wave roles (all eight compute GRU1 and GRU2):
//   0     samples (polls F2); W_hh1 rows 0..9; W_hh2 rows 24..27 in VGPRs
//   1, 2  fc1 rows 8h..8h+7 (h = w − 1) from the polled y, weights in VGPRs; W_hh2 LDS rows
//   3, 4  fc2 rows 8h..8h+7 (h = w − 3) from the polled f1 + their fc3 partials; W_hh1 rows;
//         wave 4 then gathers a quarter of the next step's GRU1 terms
//   5..7  W_hh2 rows 8(w − 5)..+7 in VGPRs; W_hh1 rows (5, 7), the h2 gather (6)
constexpr int kXWaveFc1 = 1, kXWaveFc2 = 3;
constexpr int kXH2RegRows = 28;     // W_hh2 rows 0..27 in VGPRs, 28..47 in LDS
constexpr int kXRing = 4;           // steps of conditioning terms / sampler noise in LDS
constexpr int kXNoise = 16;         // 11 MoL sampler terms, padded

// Conditioning terms of one step for one workgroup (columns of the terms GEMM), floats:
//   [0,48) P1 = W_ih1·cI, [48,96) P2 = W_ih2·[cI; a2]   (index u·3 + gate, u = local unit)
//   [96,112) cI of the own units, [112,128) V1 = W1[:, R:]·a3 + b1, [128,144) V2 = W2[:, F:]·a4 + b2
enum XTerm { XT_P1 = 0, XT_P2 = 48, XT_CI = 96, XT_V1 = 112, XT_V2 = 128, kXTerms = 160 };

// Hand-off vectors of one XCD (granules {tag = step + 1, value}, plain stores that stay in the
// XCD's L2, sc1 polls).  S (the GRU1 terms) is double-buffered by step parity.
enum XHop { XH_Y = 0, XH_F1 = 1, XH_F2 = 2, XH_H2 = 3, XH_S0 = 4, XH_S1 = 5, kXHops = 6 };
constexpr int kXF2Line = 32;        // granules per workgroup in the partial-logit vector
constexpr long long kXHopStride = 4096;            // granules per hop region (≥ 4·512, 32·32)
constexpr long long kXXcdStride = kXHops * kXHopStride + 512;   // granules per XCD

// Per-workgroup weight slab (floats), all rows natural (512 contiguous):
struct XcdSlab {
    int wih2;    // [8 waves][6 rows (2q + i)][512]   W_ih2[:, :R] gate q of unit 2w + i
    int w1;      // [16][512]                           fc1 rows 16c + r (y part)
    int w2;      // [16][512]                           fc2 rows 16c + r (f1 part)
    int whh2;    // [48][512]   W_hh2 rows u·3 + q (rows < kXH2RegRows in VGPRs, the rest LDS)
    int whh1;    // [48][512]                           W_hh1 rows u·3 + q (LDS-resident)
    int w3;      // [16][32]                            W3[j][16c + r] (j ≥ 30: 0)
    int q1a;     // [3][512]                            W_ih1·W_I[:, 0], gate-major (all units)
    int cst;     // [kXCst] small vectors, copied to LDS (XCst offsets)
    int total;
};

// Small per-workgroup vectors (LDS-resident), offsets within the cst block
enum XCst { XC_Q2 = 0, XC_BIH1 = 48, XC_BHH1 = 96, XC_BIH2 = 144, XC_BHH2 = 192, XC_WI0 = 240, XC_B3 = 256, kXCst = 288 };
//   q2 = W_ih2[:, :R]·W_I[:, 0] (own units), biases of both GRUs (own units, u·3 + q), W_I[:, 0]
//   of the own units, b3 (padded to 32)

// Per-workgroup state carried between time chunks (floats):
// [h1 512 | sg 2048 (terms of the next step) | gh2 48 | h2own 16 | x | pad]
constexpr int kXStateW = 512 + 2048 + 48 + 16 + 16;

struct XcdArgs {
    const float *slab;            // [kXcdWgs][slab.total]
    const float *terms;           // [Lc + 1][nb][kXcdWgs·kXTerms], row (t - t0)·nb + k
    const float *noise;           // [L][Bt][11] or nullptr (Philox)
    float *out;                   // [Bt][L]
    float *state;                 // [nb][kXcdWgs][kXStateW]
    unsigned long long *xg;       // [nb][kXXcdStride] granules
    int *members;                 // [kXcds] arrival counters (zeroed before the launch)
    int *ctl;                     // [0] abort, [1] code, [2] step, [3] hop, [4] wg
    unsigned long long seed;
    long long row0;               // global row id of XCD 0's row (Philox key: row0 + k)
    long long timeout_ticks;
    int L, t0, Lc, Bt, b0, nb;
    XcdSlab s;
    unsigned *dbg;                // [nb·32][dbg_steps][kStamps] or nullptr
    int dbg_steps;
};

struct XcdLds {
    int whh1, whh2, h1, h2, sg, w3, f2x, ring, nz, gh2, cst, xs, misc, total;
};

__host__ __device__ inline XcdLds xcd_lds_layout() {
    XcdLds l;
    int o = 0;
    // the small per-step arrays first (offsets < 64 KiB: lane address + instruction immediate)
    l.h1 = o;    o += 512;
    l.h2 = o;    o += 512;
    l.sg = o;    o += 4 * 512;                // GRU1 terms of all units for the coming step
    l.w3 = o;    o += kXFcRows * 32;          // fc3 columns of the own f2 rows (waves 3, 4)
    l.f2x = o;   o += 64;                     // wave 4's fc3 partials, handed to wave 3: (value, tag) pairs
    l.ring = o;  o += kXRing * kXTerms;
    l.nz = o;    o += kXRing * kXNoise;
    l.gh2 = o;   o += 48;                     // W_hh2·h2 of the own units for the next step
    l.cst = o;   o += kXCst;
    l.xs = o;    o += 4;                      // x, by step parity
    l.misc = o;  o += 8;                      // [0] abort flag, [1] member index, step flags (step + 1):
                                              // [2] h2 gathered, [3] (unused), [4] y gathered, [5] f1 gathered
    l.whh1 = o;  o += 48 * 512;
    l.whh2 = o;  o += (48 - kXH2RegRows) * 512;
    l.total = o;
    return l;
}

}  // namespace wrnn
