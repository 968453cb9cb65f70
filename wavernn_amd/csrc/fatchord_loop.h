// Shared between the host launcher (capi.cpp) and the device code (fatchord_loop.hip).
#pragma once
#include <stdint.h>

namespace wrnn {

// Wave roles.  vmcnt is in-order per wave, so a wave that polls hand-off granules must not
// have slow loads (next step's conditioning) or its own publish stores outstanding:
//   wave  0    polls (gather); computes only when a stage has more than 3 work items
//   waves 1-3  compute + publish
//   wave  4    loader: LDS-DMA of step t+1's record, Philox noise, output stores.  It never
//              reads LDS while its DMA is in flight (hipcc would drain vmcnt before the read).
constexpr int kCompute = 256;          // waves 0..3
constexpr int kWaves = kCompute / 64;
constexpr int kThreads = kCompute + 64;
constexpr int kLoaderWave = 4;
constexpr int kPollThreads = 64;
constexpr int kGatherMax = 8;          // granules per polling lane per hand-off (generic kernels)
constexpr int kClsPerLaneMax = 8;      // RAW softmax classes per lane (n_classes <= 512)
constexpr int kTermsPerUnit = 4;       // GRU1 terms exchanged per unit: S_r, S_z, Gi_n, Gh_n
constexpr int kHops = 7;
constexpr int kOverRead = 4096;        // granules a gather may read past its vector (padding)

// Hand-off vectors.  Q1 is exchanged once (prologue); S0/S1 carry the GRU1 terms of step t in
// buffer t & 1 (double-buffered: a workgroup can run at most one step ahead of another).
enum Hop { HOP_Q1 = 0, HOP_H2 = 1, HOP_F1 = 2, HOP_F2 = 3, HOP_LOGITS = 4, HOP_S0 = 5, HOP_S1 = 6 };

// Per-workgroup slab offsets (floats) of the resident weights.
struct SlabLayout {
    int wih1, whh1, wih2, whh2, bih1, bhh1, bih2, bhh2, w1, b1, w2, b2, w3, b3, wi0, total;
};

struct LoopArgs {
    const float *slab;            // [G][slab.total]
    const float *cI;              // [L][Bc][R]   I-layer conditioning projection (+bias)
    const float *cond;            // [L][Bt][CD]  mel ‖ aux
    const float *noise;           // [L][Bt][NK] or nullptr (Philox)
    float *out;                   // [Bt][L]
    int32_t *labels;              // [Bt][L] or nullptr
    unsigned long long *xg;       // [kHops][reps][rep_stride] granules {tag:32 | value:32}
    int *ctl;                     // [0] abort, [1] error code, [2] step, [3] hop, [4] wg
    unsigned long long seed;
    long long row0;               // global row id of chunk row 0 (Philox key)
    long long timeout_ticks;      // s_memrealtime ticks (100 MHz)
    int L, Bc, Bt, b0;
    int R, F, A, CD, feat, NC, NK, mol;
    int U, UF, UC, G, NMAX;
    SlabLayout s;
    int delay_poll;               // pollers wait for this WG's own publish before polling
    int reps;                     // replicas of every hand-off vector (consumer w polls w % reps)
    long long rep_stride;         // granules between replicas
    // diagnostics (WRNN_DEBUG_STAMPS): per-stage s_memrealtime stamps, [G][dbg_steps][kStamps]
    unsigned *dbg;
    int dbg_steps;
};
constexpr int kStamps = 16;

// Dynamic-LDS layout (floats) for Bc rows; shared by host sizing and the kernel.
struct LdsLayout {
    int slab, h1, h2, xa, f1, f2, lg, pre, pc, q, sg, q1a, xprev, lbl, flag, stamp, total;
    int ncp, pp, pcu;
};

__host__ __device__ inline int round4(int x) { return (x + 3) & ~3; }

// Per (row, unit) precomputed terms, kept in LDS between the stage that makes them (off the
// critical path, while a hand-off is in flight) and the stage that consumes them.
enum PcSlot { PC_P2 = 0, PC_GH2 = 3, PC_V1 = 6, PC_V2 = 7, PC_N = 8 };

__host__ __device__ inline LdsLayout lds_layout(int slab_total, int Bc, int R, int F, int A, int NC, int NK,
                                               int U, int UF) {
    LdsLayout l;
    l.ncp = round4(NC);
    l.pp = round4(R + 3 * A + NK);
    l.pcu = (U > UF ? U : UF);                 // pc entries per row (unit u and fc row u share)
    int o = 0;
    l.slab = o;  o += round4(slab_total);
    l.h1 = o;    o += Bc * R;
    l.h2 = o;    o += Bc * R;
    l.xa = o;    o += Bc * (R + A);            // [x_I + h1 | a3]
    l.f1 = o;    o += Bc * F;
    l.f2 = o;    o += Bc * F;
    l.lg = o;    o += Bc * l.ncp;
    l.pre = o;   o += 3 * Bc * l.pp;           // ring of 3 step records
    l.pc = o;    o += Bc * l.pcu * PC_N;
    l.q = o;     o += round4(6 * U);           // Q1, Q2: W_ih·W_I[:,0] per gate row (own units)
    l.sg = o;    o += Bc * R * kTermsPerUnit;  // GRU1 terms of ALL units for the coming step
    l.q1a = o;   o += round4(3 * R);           // Q1 of all units, gate-major
    l.xprev = o; o += round4(Bc);
    l.lbl = o;   o += round4(Bc);
    l.flag = o;  o += 4 + kHops * kWaves + 4;  // abort word + per-hop, per-wave publish flags
    l.stamp = o; o += 2 * kStamps;
    l.total = o;
    return l;
}

}  // namespace wrnn
