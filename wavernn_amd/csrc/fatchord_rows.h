// Shared between the host launcher (capi.cpp) and fatchord_rows.hip: the multi-row
// (fold-batched) variant of the sample loop.
#pragma once
#include <stdint.h>

#include "fatchord_loop.h"

namespace wrnn {

// Activations of all rows move through HBM as bulk hand-offs: producers store their slice with
// sc1 stores, drain them (s_waitcnt vmcnt(0) per storing wave), pass a workgroup barrier, and one
// lane stores the step into the workgroup's flag; consumers poll every producer's flag, then
// load the rows with sc1 LDS-DMA (MI355X_MICROARCH.md "Valid forms", first table row).
constexpr int kRowsHops = 5;        // h1, h2, f1, f2, logits (RAW)
// Granule hand-offs (small row counts): a stage's activations travel as 8-byte {tag, value}
// granules that the loader waves poll straight into the LDS tile — no store drain, barrier, flag
// or post-flag DMA.  kRowsGranNG loads per loader lane per poll round (4 loader waves).
constexpr int kRowsGranNG = 16;
constexpr int kRowsGranPad = kRowsGranNG * 256;   // granules a poll round may read past a vector
constexpr int kFlagStride = 32;     // uints between two producers' flags (one 128-B line each)
constexpr int kFlagSlots = 256;     // producer slots per hop: >= G, fixed so polls may over-read
constexpr int kRowsMax = 256;       // rows per launch (x hand-off: <= 4 granules per polling lane)
constexpr int kXReps = 8;           // replicas of the x granules
constexpr int kXRepStride = 8192;   // granules between x replicas (64 KiB)
constexpr int kDotEngines = 16;     // 16-lane dot engines: 4 compute waves x 4 DPP rows
// fatchord_rows_kernel: 12 waves, 0-7 compute (two per SIMD: one wave alone issues a VALU op
// every 4 cycles, two interleave to the 2-cycle rate, MI355X_MICROARCH.md cycle table), 8-11 load.
// A stage's activation tiles are LDS-DMA'd by all four loader waves (one wave streams a fresh tile
// at only ~13-15 GB/s, handoff-payload row; at 115 rows that alone made each stage DMA-bound).
// Wave 8 also polls the flags, streams the terms/draws and feeds the samplers.
constexpr int kRowsComputeWaves = 8;
constexpr int kRowsCompute = 64 * kRowsComputeWaves;
constexpr int kRowsEngines = 4 * kRowsComputeWaves;   // 16-lane dot engines
constexpr int kRowsLoaders = 4;
constexpr int kRowsLead = kRowsComputeWaves;           // first loader wave
constexpr int kRowsThreads = kRowsCompute + 64 * kRowsLoaders;

enum RowsHop { RH_H1 = 0, RH_H2 = 1, RH_F1 = 2, RH_F2 = 3, RH_LG = 4 };

// Per-workgroup resident weights (floats).  Only the parts that multiply per-step state are
// here; everything linear in the conditioning is in the precomputed terms.
//
// Block-sparse GRU weights (BASELINE config 4, wavernn_amd/pruning.py): with U = 4 a workgroup
// owns one 4-row block-row per gate of W_ih2[:, :R], W_hh1, W_hh2; only its nonzero 4x4 blocks
// are kept — sp: [3 matrices][3 gates][nbmax][16] (row-major 4x4), spc: block-column index per
// block (int bits), spn: [3][3] block counts.  The dense wih2/whh1/whh2 regions are then empty.
struct RowsSlab {
    int wih2, whh1, whh2, w1, w2, w3, b3, bih1, bhh1, bih2, bhh2, q1, q2, q3, sp, spc, spn, nbmax;
    int body;      // floats before the MoL head (which is last); RAW: == total
    int total;
};
enum SparseMat { SP_WIH2 = 0, SP_WHH1 = 1, SP_WHH2 = 2 };

// Precomputed per (step, row, workgroup) terms, NT floats: [P1 3U | P2 3U | V1c UF | V2 UF | pad]
//   P1  = W_ih1[g·R+j]·cI             P2 = W_ih2[g·R+j]·[cI; a2]
//   V1c = W1[r]·[cI; a3] + b1[r]      V2 = W2[r, F:]·a4 + b2[r]
__host__ __device__ inline int rows_terms(int U, int UF) { return round4(6 * U + 2 * UF); }

// Carried per-row state of a workgroup's own units (floats within a row's SW block)
enum RowsState { RS_H1 = 0 };   // h1o U | h2o U | GH1 3U | GH2 3U | V1h UF
__host__ __device__ inline int rows_state_width(int U, int UF) { return round4(8 * U + UF); }

struct RowsArgs {
    const float *slab;            // [G][s.total]
    const float *terms;           // [Lc][B][G·NT] precomputed terms of this launch's steps
    const float *noise;           // [L][Bt][NK] or nullptr (Philox)
    float *out;                   // [Bt][L]
    int32_t *labels;              // [Bt][L] or nullptr
    float *act;                   // [kRowsHops][2][B][KA] activations, parity = step & 1
    unsigned *flags;              // [kRowsHops][kFlagSlots][kFlagStride]
    unsigned long long *xg;       // [kXReps][kXRepStride] x granules {tag | value}
    unsigned long long *gact;     // granule mode: [kRowsHops][gstride] {tag = step + 1 | value}; else nullptr
    long long gstride;            // granules per hop (>= B·KA + kRowsGranPad)
    unsigned long long *gf2;      // bulk mode, MoL: the f2 hop as granules [B][F] (samplers poll their
                                  // row directly instead of all flags + DMA); else nullptr
    float *state;                 // [G][B][SW] carried state, then x [B]
    int *ctl;                     // as LoopArgs::ctl
    unsigned long long seed;
    long long row0;
    long long timeout_ticks;
    int L, t0, Lc;                // total steps, first step of this launch, steps in this launch
    int B, Bt, b0;                // rows in this launch, rows in out/noise, first row
    int R, F, A, NC, NK, mol, U, UF, UC, G, NT, TB, KA;
    RowsSlab s;
    unsigned *dbg;                // WRNN_DEBUG_STAMPS: [G][dbg_steps][kStamps] s_memrealtime per stage
    int dbg_steps;
    int head_lds;                 // MoL: 1 = head in LDS, 0 = samplers read it from HBM (workgroup 0's slab)
    int gw;                       // 1 = streamed weights: the slab stays in HBM (weights exceed LDS)
};

// The per-group fields of a second row group sharing the launch (fatchord_rows.hip)
struct RowsGroup {
    const float *terms;
    float *act;
    unsigned *flags;
    unsigned long long *xg;
    unsigned long long *gact;
    unsigned long long *gf2;
    float *state;
    long long row0;
    int B, b0;
    unsigned *dbg;
};

struct RowsLds {
    int slab, tile, st, x, ring, lg, nz, flag, total;
    int SW, KT, NS, ncp, nkp;
};

__host__ __device__ inline RowsLds rows_lds_layout(int slab_total, int B, int TB, int R, int F, int NC, int NK,
                                                   int U, int UF, int G) {
    RowsLds l;
    l.SW = rows_state_width(U, UF);
    l.KT = round4(R > F ? (R > NC ? R : NC) : (F > NC ? F : NC));
    l.NS = (B + G - 1) / G;                    // rows this workgroup samples (b = w, w + G, ...)
    l.ncp = round4(NC);
    l.nkp = round4(NK);
    const int NT = rows_terms(U, UF);
    const int tr = 2 * TB > l.NS ? 2 * TB : l.NS;   // two tiles (double-buffered DMA)
    int o = 0;
    l.slab = o;  o += round4(slab_total);
    l.tile = o;  o += tr * l.KT;
    l.st = o;    o += B * l.SW;
    l.x = o;     o += round4(B);
    l.ring = o;  o += 2 * B * NT;              // terms of steps t, t+1
    l.lg = o;    o += l.NS * l.ncp;
    l.nz = o;    o += 2 * l.NS * l.nkp;        // sampler draws of steps t, t+1
    l.flag = o;  o += 8;
    l.total = o;
    return l;
}

}  // namespace wrnn
