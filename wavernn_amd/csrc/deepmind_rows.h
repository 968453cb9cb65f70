// Shared between capi.cpp and deepmind_rows.hip: the dual-softmax (deepmind_version.py) loop.
#pragma once
#include <stdint.h>

#include "fatchord_rows.h"

namespace wrnn {

// Bulk hand-offs of one step (flags + LDS-DMA, as the fatchord rows kernel) and the two
// x hand-offs of the sampled labels (tagged granules).
enum DmHop { DH_HC = 0, DH_O1 = 1, DH_LC = 2, DH_HF = 3, DH_O3 = 4, DH_LF = 5, kDmHops = 6 };

// 8 waves: 0-3 compute (16 dot engines), 4-7 split each tile's LDS-DMA; wave 4 also polls flags
constexpr int kDmLoaders = 4;
constexpr int kDmThreads = kCompute + 64 * kDmLoaders;
// Granule hand-offs (as fatchord_rows.h) while a group's hop vector holds <= kDmGranMax values:
// a stage's first tile is polled by all eight waves (the compute waves would only wait at the
// barrier), 16 loads per lane per round; later tiles by the four loader waves.
constexpr int kDmGranNG = 16;
constexpr int kDmGranPad = kDmGranNG * kDmThreads;

// Per-workgroup resident weights (floats).  Workgroup w owns coarse units j = w·U + u and the
// fine units S + j (u < U) — their u/r/e rows of R (3H × H, no bias, deepmind_version.py:16),
// split in the generate() order [cu | fu | cr | fr | ce | fe] (:116-119) — plus UO rows of each
// output layer O1..O4 (:19-22), its rows of I_coarse (2 inputs) and I_fine (3 inputs) (:25-26)
// and the gate biases (:29-31).
struct DmSlab {
    int rw;        // [6][U][H]: (half·3 + gate)·U + u, half 0 = coarse unit, 1 = fine unit
    int o1, o1b, o2, o2b, o3, o3b, o4, o4b;   // [UO][S] / [UO][S] / [UO2][S] / [UO2][S] (+ biases)
    int ic, if_;   // [3][U][2], [3][U][3]
    int bu, br, be;   // [2][U] (coarse, fine)
    int total;
};

struct DmArgs {
    const float *slab;            // [G][s.total]
    const float *noise;           // [L][Bt][2Q] (q_coarse | q_fine) or nullptr (Philox)
    float *out;                   // [Bt][L] combined 16-bit sample as float (utils/dsp.py:33)
    int32_t *labels;              // [Bt][L] combined sample as int, or nullptr
    float *act;                   // [kDmHops][2][B][KA]
    unsigned *flags;              // [kDmHops][kFlagSlots][kFlagStride]
    unsigned long long *xg;       // [2 (coarse, fine)][kXReps][kXRepStride]
    unsigned long long *gact;     // granule mode: [kDmHops][gstride] {tag = step + 1 | value}; else nullptr
    long long gstride;
    float *state;                 // [G][B][SW] carried state, then prev labels [2][B]
    int *ctl;
    unsigned long long seed;
    long long row0;
    long long timeout_ticks;
    int L, t0, Lc, B, Bt, b0;
    int H, S, Q, U, UO, UO2, G, TB, KA;
    DmSlab s;
    int gw;                       // 1 = streamed weights: the slab stays in HBM (exceeds LDS)
};

// The per-group fields of a second row group sharing the launch (as RowsGroup, fatchord_rows.h)
struct DmGroup {
    float *act;
    unsigned *flags;
    unsigned long long *xg;
    unsigned long long *gact;
    float *state;
    long long row0;
    int B, b0;
};

// Per-row state of a workgroup's own units: hc U | hf U | Rh[2 parities][2 halves of h][6][U]
__host__ __device__ inline int dm_state_width(int U) { return round4(2 * U + 24 * U); }

struct DmLds {
    int slab, tile, st, pc, pf, cn, cs, nz, flag, total;
    int SW, KT, NS, nkp;
};

__host__ __device__ inline DmLds dm_lds_layout(int slab_total, int B, int TB, int S, int Q, int U, int G) {
    DmLds l;
    l.SW = dm_state_width(U);
    l.KT = round4(S > Q ? S : Q);
    l.NS = (B + G - 1) / G;
    l.nkp = round4(2 * Q);
    const int tr = 2 * TB > l.NS ? 2 * TB : l.NS;
    int o = 0;
    l.slab = o;  o += round4(slab_total);
    l.tile = o;  o += tr * l.KT;
    l.st = o;    o += B * l.SW;
    l.pc = o;    o += round4(B);               // previous coarse / fine labels (as floats)
    l.pf = o;    o += round4(B);
    l.cn = o;    o += round4(B);               // c_t of every row (after the coarse x hop)
    l.cs = o;    o += round4(l.NS);            // c_t of this workgroup's sampled rows
    l.nz = o;    o += 2 * l.NS * l.nkp;        // draws of steps t, t+1 for the sampled rows
    l.flag = o;  o += 8;
    l.total = o;
    return l;
}

}  // namespace wrnn
