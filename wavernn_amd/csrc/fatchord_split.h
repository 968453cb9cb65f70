// Shared between the host launcher (capi.cpp) and fatchord_split.hip: the role-split latency
// kernel for one MoL row (the BASELINE headline, batch 1).
#pragma once
#include <stdint.h>

#include "fatchord_loop.h"

namespace wrnn {

constexpr int kSplitUnits = 4;       // GRU units (both GRUs) per GRU workgroup
constexpr int kSplitFcRows = 16;     // fc1 and fc2 rows per FC workgroup (one per 16-lane engine)
constexpr int kSplitTerms = 32;      // conditioning terms per workgroup per step (terms-GEMM columns)
constexpr int kSplitRing = 4;        // steps of terms / sampler noise held in LDS
constexpr int kSplitNoise = 12;      // 11 MoL sampler terms, padded
constexpr int kYLine = 16;           // granules (one 128-B line) per GRU workgroup in the y vector

// Hand-off vectors (granules {tag = step + 1, value}).  H2 and the GRU1 terms are double-
// buffered by step parity; Y, F1, F2 are not (the step's dependency chain orders their reuse).
enum SplitHop { SH_Y = 0, SH_F1 = 1, SH_F2 = 2, SH_H2A = 3, SH_H2B = 4, SH_S0 = 5, SH_S1 = 6, kSplitHops = 7 };

// Terms of one step (columns of the conditioning GEMM), per role:
//   GRU workgroup: [0,12) P1 = W_ih1·cI, [12,24) P2 = W_ih2·[cI; a2]  (index u·3 + gate),
//                  [24,28) cI of its own units (identity rows: exact)
//   FC workgroup:  [0,16) V1c = W1[:, R:]·a3 + b1,  [16,32) V2 = W2[:, F:]·a4 + b2
enum SplitTerm { ST_P1 = 0, ST_P2 = 12, ST_CI = 24, ST_V1 = 0, ST_V2 = 16 };

// Slabs (floats).  fc3 is split by its input columns: FC workgroup f holds W3[:, 16f..16f+15]
// (w3p[e·32 + j] = W3[j][16f + e]) and publishes the 30 partial logits of its 16 f2 rows; the
// GRU workgroups keep only b3 for the sum.
struct SplitGruSlab {
    int b3, wih2, whh1, whh2, q1a, q2, wi0, bih1, bhh1, bih2, bhh2, total;
};
struct SplitFcSlab {
    int w3p, w1, w2, total;
};
constexpr int kSplitLogitLine = 32;   // granules per FC workgroup in the partial-logit vector

// Per-workgroup state carried between time chunks (floats):
// [h1 R | h2 R | GRU1 terms 4R | gh2 24 | h2own 4 | x | pad]
__host__ __device__ constexpr int split_state_w(int R) { return (2 + kTermsPerUnit) * R + 32; }

struct SplitArgs {
    const float *gslab;           // [Gg][gs.total]
    const float *fslab;           // [Gf][fs.total]
    const float *terms;           // [Lc + 1][(Gg + Gf)·kSplitTerms], row = t - t0
    const float *noise;           // [L][Bt][11] or nullptr (Philox)
    float *out;                   // [Bt][L]
    float *state;                 // [Gg + Gf][kSplitStateW(R)]
    unsigned long long *xg;       // [kSplitHops][reps][rep_stride]
    int *ctl;                     // [0] abort, [1] code, [2] step, [3] hop, [4] wg
    unsigned long long seed;
    long long row0;               // global row id (Philox key)
    long long timeout_ticks;
    long long rep_stride;         // granules between replicas
    int L, t0, Lc, Bt, b0;
    int Gg, Gf, reps;
    SplitGruSlab gs;
    SplitFcSlab fs;
    unsigned *dbg;                // [G][dbg_steps][kStamps] or nullptr
    int dbg_steps;
};

struct SplitLds {
    int slab, va, vb, f2, sg, ring, nz, gh2, gh1, h2own, xprev, flag, stamp, total;
};

__host__ __device__ inline SplitLds split_lds_layout(int slab_total, int R, int F) {
    SplitLds l;
    int o = 0;
    l.slab = o;  o += round4(slab_total);
    l.va = o;    o += round4(R > F ? R : F);     // GRU: h1          FC: y = x_I + h1 + h2
    l.vb = o;    o += round4(R > F ? R : F);     // GRU: h2 (all)    FC: f1
    l.f2 = o;    o += 32;                         // FC: its own 16 f2 rows
    l.sg = o;    o += kTermsPerUnit * R;          // GRU1 terms of all units for the coming step
    l.ring = o;  o += kSplitRing * kSplitTerms;
    l.nz = o;    o += kSplitRing * kSplitNoise;
    l.gh2 = o;   o += 2 * 12;                     // W_hh2·h2 of own units, by step parity
    l.gh1 = o;   o += 12;
    l.h2own = o; o += 4;
    l.xprev = o; o += 4;                          // x_t, by step parity
    l.flag = o;  o += 4;
    l.stamp = o; o += 2 * kStamps;
    l.total = o;
    return l;
}

}  // namespace wrnn
