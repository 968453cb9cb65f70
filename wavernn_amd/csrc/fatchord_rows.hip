// fatchord_rows.hip — persistent CDNA4 kernel for MANY rows of the WaveRNN sample loop.
//
// The fold-batched generate() (models/fatchord_version.py:186-188, fold_with_overlap :293-340)
// runs B independent rows (folds, or utterances) through the same loop (:201-241).  The latency
// kernel (fatchord_loop.hip) keeps every row's activations in LDS and exchanges them as tagged
// granules, which fits ~1 row next to the weights.  This kernel keeps only the weights and a
// few floats of per-row state in LDS and moves whole activation matrices [B][512] through HBM:
//
//   * grid = G workgroups (one per CU); workgroup w owns GRU units [w·U, w·U+U), fc1/fc2 rows
//     [w·UF, …) and (RAW) fc3 rows [w·UC, …), as in the latency kernel;
//   * every term that depends only on the conditioning (P1, P2, the conditioning part of fc1,
//     V2) was computed for all steps by one fp32 GEMM before the launch (capi.cpp: rocBLAS),
//     so a workgroup streams NT = 16 floats per row-step of its own terms;
//   * each stage ends in a bulk hand-off (fatchord_rows.h): sc1 stores → vmcnt(0) → barrier →
//     flag; consumers poll all G flags and LDS-DMA the rows (sc1) tile by tile;
//   * sampling is distributed by row: workgroup w samples rows w, w+G, … (MoL: fc3 + sampler;
//     RAW: sampler over the gathered logits) and hands x to everyone as tagged granules.
//
// Per step:  GRU1 own units (all rows) → [h1] → GRU2 (W_ih2[:, :R]·h1) → [h2] → fc1 → [f1] →
//            fc2 → [f2] → (RAW: fc3 → [logits]) → sample (row-distributed) → [x] → next step.
// Off the critical path (after a stage's flag, overlapping the next hand-off):
//   GH1_{t+1} = W_hh1·h1_t and V1h = W1[:, :R]·h1_t (on the h1 tiles), GH2_{t+1} = W_hh2·h2_t.
// Arithmetic is fp32 throughout, in the same re-associated forms as the latency kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fatchord_rows.h"
#include "rows_device.h"

namespace wrnn {

// cache policy of the stage-tile LDS-DMA: 0 = plain behind an agent acquire, 16 = sc1
#ifndef WRNN_TILE_CPOL
#define WRNN_TILE_CPOL 16
#endif
constexpr int kTileCpol = WRNN_TILE_CPOL;

// kRF = 512 instantiates the shipped dims (rnn_dims = fc_dims = 512) with compile-time dot
// lengths; 0 = runtime dims.  SPARSE: block-sparse GRU weights (one 4-unit block-row per gate,
// U = 4), the GRU matvecs run one engine per activation row over the nonzero blocks.
//
// Row groups: workgroups [0, G0) run argument set a0, [G0, 2·G0) set a1 — two independent
// instances of the loop (own rows, buffers, flags) in one launch.  With B large the activation
// broadcast (every workgroup DMAs every row of every stage) is what limits a stage; two groups of
// G/2 workgroups, each holding twice the weight rows, halve the rows each workgroup streams.
//
// GW (streamed weights): the workgroup's slab stays in HBM and every weight read is a global load
// (L2 / Infinity-Cache served after the first step).  For models whose dense weights exceed the
// grid's LDS (e.g. rnn 896 unpruned: 32 MB of loop weights), so the drop-in accepts every size the
// reference constructor does (models/fatchord_version.py:93-129); LDS then holds only row state.
template <bool MOL, int kRF, bool SPARSE, bool GW>
__global__ __launch_bounds__(kRowsThreads) void fatchord_rows_kernel(RowsArgs a, RowsGroup g1, int G0) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, row = lane >> 4;
    const bool grp1 = (int)blockIdx.x >= G0;
    if (grp1) {   // field by field (uniform selects; a dynamically chosen struct would go to scratch)
        a.terms = g1.terms;
        a.act = g1.act;
        a.flags = g1.flags;
        a.xg = g1.xg;
        a.gact = g1.gact;
        a.gf2 = g1.gf2;
        a.state = g1.state;
        a.row0 = g1.row0;
        a.B = g1.B;
        a.b0 = g1.b0;
        a.dbg = g1.dbg;
    }
    const int w = (int)blockIdx.x - (grp1 ? G0 : 0);
    const int R = kRF ? kRF : a.R, F = kRF ? kRF : a.F, NC = a.NC, NK = a.NK, U = a.U, UF = a.UF, UC = a.UC, G = a.G, B = a.B;
    const int NT = a.NT, TB = a.TB, KA = a.KA;
    const int slab_lds = GW ? 0 : (MOL && !a.head_lds) ? a.s.body : a.s.total;   // floats resident in LDS
    const RowsLds ll = rows_lds_layout(slab_lds, B, TB, R, F, NC, NK, U, UF, G);
    const RowsSlab &s = a.s;
    const float *S = GW ? a.slab + (size_t)w * s.total : smem + ll.slab;
    // MoL head [NC][F] then bias [NC]: LDS, or (large B) the HBM copy in workgroup 0's slab
    const float *head = (MOL && !a.head_lds && !GW) ? a.slab + a.s.w3 : S + a.s.w3;
    const int *spc = reinterpret_cast<const int *>(S + a.s.spc);     // sparse: block columns, counts
    const int *spn = reinterpret_cast<const int *>(S + a.s.spn);
    float *tile = smem + ll.tile, *st = smem + ll.st, *xs = smem + ll.x, *ring = smem + ll.ring;
    float *lgs = smem + ll.lg, *nzs = smem + ll.nz;
    int *abort_flag = reinterpret_cast<int *>(smem + ll.flag);
    const int SW = ll.SW, NS = ll.NS;
    const int O_H2 = U, O_GH1 = 2 * U, O_GH2 = 5 * U, O_V1 = 8 * U;   // offsets in a row's state
    const int Uv = max(0, min(U, R - w * U));
    const int UFv = max(0, min(UF, F - w * UF));
    const int UCv = MOL ? 0 : max(0, min(UC, NC - w * UC));
    const bool loader = wave >= kRowsLead;             // waves 8-11: tile DMA
    const bool lead = wave == kRowsLead;               // wave 8: flag polls, terms, draws, samplers
    const bool compute = !loader;
    int *go = abort_flag + 1;                          // LDS: wave 8 → other loaders, "flags seen"
    const int eng = wave * 4 + row;                    // dot engine of this lane (compute waves)
    const size_t hop_sz = (size_t)2 * B * KA;
    unsigned *dbgw = a.dbg ? a.dbg + (size_t)w * a.dbg_steps * kStamps : nullptr;
#define RSTAMP(k)                                                                                   \
    do {                                                                                            \
        if (dbgw && tid == 0 && tl < a.dbg_steps)                                                  \
            dbgw[(size_t)tl * kStamps + (k)] = (unsigned)__builtin_amdgcn_s_memrealtime();          \
    } while (0)
    auto actp = [&](int hop, int t) { return a.act + hop * hop_sz + (size_t)(t & 1) * B * KA; };
    auto flagp = [&](int hop) { return a.flags + (size_t)hop * kFlagSlots * kFlagStride; };
    const bool gran = a.gact != nullptr;
    auto signal = [&](int hop, int t) {                // after every storing wave's vmcnt(0) + a barrier
        if (!gran && tid == 0)
            __hip_atomic_store(flagp(hop) + w * kFlagStride, (unsigned)t + 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };
    // one activation value of row b, column k of hop `hop` at step t: a granule, or an sc1 store
    // into the bulk matrix `bulk` (row stride K)
    auto put = [&](int hop, float *bulk, int b, int K, int k, int t, float v) {
        if (gran) publish(a.gact + (size_t)hop * a.gstride + (size_t)b * K + k, (uint32_t)t + 1u, v);
        else if (MOL && hop == RH_F2 && a.gf2) publish(a.gf2 + (size_t)b * K + k, (uint32_t)t + 1u, v);
        else store_sc1(bulk + (size_t)b * K + k, v);
    };
    // granule mode: rows [r0, r0 + nr) of hop `hop` (step t) polled by the four loader waves
    // straight into an LDS tile, rows packed at stride K like the bulk DMA's
    auto gran_tile = [&](float *dst, int hop, int K, int r0, int nr, int t) {
        const int lid = (wave - kRowsLead) * 64 + lane;
        auto st_ = [&](int b, int j, float v) { dst[b * K + j] = v; };
        gather_chunked<kRowsGranNG, 256, decltype(st_)>(a.gact + (size_t)hop * a.gstride + (size_t)r0 * K, nr * K, K,
                                                        (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t, hop, abort_flag,
                                                        lid, st_);
    };
    // LDS-DMA (sc1) of n floats (contiguous rows) from src into dst, issued by one wave
    auto dma = [&](float *dst, const float *src, int n) {
        for (int c = 0; c < n; c += 256)
            if (c + lane * 4 < n)
                __builtin_amdgcn_global_load_lds(WRNN_GPTR(src + c + lane * 4), WRNN_LPTR(dst + c), 16, 0, 16);
    };
    // the same split over the four loader waves (1 KiB pieces, round robin).  Plain (L2-cached)
    // loads behind the lead wave's agent-scope acquire (MI355X_MICROARCH.md "Valid forms",
    // consumer: one relaxed poll → one agent acquire → vmcnt(0) → plain loads): the 32 CUs of an
    // XCD then share one fetch of each activation line instead of each pulling it past L2.
    auto dma_part = [&](float *dst, const float *src, int n) {
        for (int c = (wave - kRowsLead) * 256; c < n; c += kRowsLoaders * 256)
            if (c + lane * 4 < n)
                __builtin_amdgcn_global_load_lds(WRNN_GPTR(src + c + lane * 4), WRNN_LPTR(dst + c), 16, 0, kTileCpol);
    };
    // draws of step t for this workgroup's sampled rows → nz slot (t & 1); MoL turned into sampler terms
    auto load_noise = [&](int t, int id, int nl) {
        float *slot = nzs + (t & 1) * NS * ll.nkp;
        for (int i = id; i < NS * NK; i += nl) {
            const int sr = i / NK, k = i - sr * NK, b = w + sr * G;
            if (b >= B) continue;
            float v = a.noise ? a.noise[((size_t)t * a.Bt + a.b0 + b) * NK + k]
                              : philox_noise(a.seed, (unsigned long long)(a.row0 + b), (uint32_t)t, (uint32_t)k, MOL);
            if (MOL) v = mol_noise_term(v, k);
            slot[sr * ll.nkp + k] = v;
        }
    };
    auto load_terms = [&](int tl, int id, int nl) {
        float4 *dst = reinterpret_cast<float4 *>(ring + (tl & 1) * B * NT);
        const int q = NT / 4;
        for (int i = id; i < B * q; i += nl) {
            const int b = i / q, k = i - b * q;
            dst[i] = reinterpret_cast<const float4 *>(a.terms + ((size_t)tl * B + b) * G * NT + (size_t)w * NT)[k];
        }
    };

    // ---- prologue: weights, carried state, terms + draws of the first step
    {
        const float4 *src = reinterpret_cast<const float4 *>(a.slab + (size_t)w * s.total);
        float4 *dst = reinterpret_cast<float4 *>(smem + ll.slab);
        if (!GW)
            for (int i = tid; i < slab_lds / 4; i += kRowsThreads) dst[i] = src[i];
        const float *cs = a.state + (size_t)w * B * SW;
        for (int i = tid; i < B * SW; i += kRowsThreads) st[i] = a.t0 > 0 ? cs[i] : 0.0f;
        const float *cx = a.state + (size_t)G * B * SW;
        for (int i = tid; i < B; i += kRowsThreads) xs[i] = a.t0 > 0 ? cx[i] : 0.0f;   // x = 0 (:196)
        if (tid == 0) {
            *abort_flag = 0;
            *go = -1;
        }
        load_terms(0, tid, kRowsThreads);
        load_noise(a.t0, tid, kRowsThreads);
    }
    __syncthreads();

    // ---- matvec stages.  A stage reads one activation matrix [B][K] tile by tile (LDS-DMA,
    // double-buffered: tile k+1 lands while tile k is computed) and runs a job list on each
    // tile: a job is one 16-lane engine's block of weight rows × up to kNX activation rows.
    // Critical and off-critical jobs of a stage share the list (critical ones first), so the
    // 16 engines stay busy and each activation row is read from HBM once per stage.
    constexpr int kNX = 4;
    auto tbuf = [&](int k) { return tile + (k & 1) * TB * ll.KT; };
    int t_cur = a.t0;                                  // step the stage driver works on
#define RSTAMP_T(k)                                                                                 \
    do {                                                                                            \
        if (dbgw && tid == 0 && t_cur - a.t0 < a.dbg_steps)                                        \
            dbgw[(size_t)(t_cur - a.t0) * kStamps + (k)] = (unsigned)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
    // Stage driver.  Wave 8 polls the hop's flags and releases the other loader waves through an
    // LDS word; the four loader waves split every tile DMA, each waiting only for its own loads;
    // the compute waves run the jobs and store their outputs (sc1), and drain those stores once,
    // before the stage's signal.  Returns false on abort.
    auto run_stage = [&](int hop, int K, auto &&jobs) -> bool {
        const float *src = actp(hop, t_cur);
        const int ntiles = (B + TB - 1) / TB;
        if (loader && gran) {
            gran_tile(tbuf(0), hop, K, 0, min(TB, B), t_cur);
        } else if (loader) {
            const int go_val = (t_cur + 1) * kRowsHops + hop;
            if (lead) {
                wait_flags(flagp(hop), G, (unsigned)t_cur + 1u, a.ctl, a.timeout_ticks, t_cur, hop, abort_flag);
                if (kTileCpol == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __hip_atomic_store(go, go_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                while (__hip_atomic_load(go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != go_val)
                    __builtin_amdgcn_s_sleep(1);
            }
            if (!*reinterpret_cast<volatile int *>(abort_flag)) dma_part(tbuf(0), src, min(TB, B) * K);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        if (hop == RH_H2) RSTAMP_T(13);
        if (*abort_flag) return false;
        unsigned long long busy = 0;                   // diagnostics: summed job / DMA time of the fc1 stage
        for (int k = 0; k < ntiles; ++k) {
            const int tb0 = k * TB, nb = min(TB, B - tb0);
            const unsigned long long c0 = dbgw ? __builtin_amdgcn_s_memrealtime() : 0;
            if (loader && k + 1 < ntiles) {
                if (gran) {
                    gran_tile(tbuf(k + 1), hop, K, tb0 + TB, min(TB, B - tb0 - TB), t_cur);
                } else {
                    dma_part(tbuf(k + 1), src + (size_t)(tb0 + TB) * K, min(TB, B - tb0 - TB) * K);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            if (compute) jobs(tbuf(k), tb0, nb);
            if (dbgw) busy += __builtin_amdgcn_s_memrealtime() - c0;
            bar();
        }
        if (dbgw && hop == RH_H2 && t_cur - a.t0 < a.dbg_steps && lane == 0 && (wave == 0 || lead))
            dbgw[(size_t)(t_cur - a.t0) * kStamps + (lead ? 8 : 5)] = (unsigned)busy;
        if (hop == RH_H2) RSTAMP_T(14);
        if (!gran) {   // bulk: every storing wave drains before the stage's signal
            if (compute) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
        }
        if (hop == RH_H2) RSTAMP_T(15);
        return true;
    };
    // job helpers: unit blocks (3 gate rows of unit u) and fc blocks (2 rows r0, r0+1)
    // (lane li of the engine ends up with activation row li & 3 of the block)
    constexpr int KI = kRF / 64;                       // chunks per lane when R = F = kRF
    auto unit_block = [&](int wbase, const float *x, int K, int nx, int u, float (&acc)[3]) {
        bdot4<3, KI>(S + wbase + u * K, U * K, x, K, nx, K / 4, li, acc);
    };
    auto fc_block = [&](int wbase, int nrows, const float *x, int K, int nx, int r0, float (&acc)[2]) {
        const int r1 = r0 + 1 < nrows ? r0 + 1 : r0;
        bdot4<2, KI>(S + wbase + r0 * K, (r1 - r0) * K, x, K, nx, K / 4, li, acc);
    };
    const int nUF2 = (UFv + 1) / 2, nUC2 = (UCv + 1) / 2;

    for (int tl = 0; tl < a.Lc; ++tl) {
        const int t = a.t0 + tl;
        t_cur = t;
        const unsigned want = (unsigned)t + 1u;
        const float *T = ring + (tl & 1) * B * NT;
        RSTAMP(0);

        // ---- GRU1 (:208-210), own units, every row
        if (compute) {
            float *h1o = actp(RH_H1, t);
            for (int i = tid; i < B * Uv; i += kRowsCompute) {
                const int b = i / Uv, u = i - b * Uv, j = w * U + u;
                const float x = xs[b];
                const float *Tb = T + b * NT;
                float *sb = st + b * SW;
                float gi[3], gh[3];
#pragma unroll
                for (int g = 0; g < 3; ++g) {
                    gi[g] = fmaf(x, S[s.q1 + g * U + u], Tb[g * U + u]) + S[s.bih1 + g * U + u];
                    gh[g] = sb[O_GH1 + g * U + u] + S[s.bhh1 + g * U + u];
                }
                const float hn = gru_gate_math(gi[0], gi[1], gi[2], gh[0], gh[1], gh[2], sb[u]);
                sb[u] = hn;
                put(RH_H1, h1o, b, R, j, t, hn);
            }
            if (!gran) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        signal(RH_H1, t);
        RSTAMP(1);

        // ---- GRU2 (:212-214): W_ih2[:, :R]·h1 + P2 + x·Q2 → h2; with GH1_{t+1} = W_hh1·h1 and
        // V1h = W1[:, :R]·h1 (the h1 part of fc1's input x = x_I + h1 + h2)
        RSTAMP(2);
        {
            float *h2o = actp(RH_H2, t);
            const bool ok = run_stage(RH_H1, R, [&](const float *tl_, int tb0, int nb) {
                // job types padded to multiples of 4 so the 4 engines of a wave never diverge:
                // [GRU2 gates | GH1 of the next step | V1h rows]; unit jobs are (unit, 4-row
                // block) dense, (row) sparse
                const int nbb = (nb + kNX - 1) / kNX, n1 = SPARSE ? nb : Uv * nbb, nj1 = round4(n1);
                const int nj2 = 2 * nj1, nj3 = nj2 + nUF2 * nbb;
                for (int jb = eng; jb < nj3; jb += kRowsEngines) {
                    if (jb < nj2) {
                        const bool crit = jb < nj1;
                        const int jj = crit ? jb : jb - nj1;
                        if (jj >= n1) continue;
                        float acc[3];
                        int u, b;
                        bool mine;
                        if (SPARSE) {
                            const int m = crit ? SP_WIH2 : SP_WHH1;
                            sparse_gates4(S + s.sp + m * 3 * s.nbmax * 16, spc + m * 3 * s.nbmax, spn + m * 3, s.nbmax,
                                          tl_ + jj * R, li, acc);
                            u = li;
                            b = tb0 + jj;
                            mine = li < Uv;
                        } else {
                            u = jj % Uv;
                            const int bb = jj / Uv, nx = min(kNX, nb - bb * kNX);
                            unit_block(crit ? s.wih2 : s.whh1, tl_ + bb * kNX * R, R, nx, u, acc);
                            b = tb0 + bb * kNX + li;
                            mine = li < nx;
                        }
                        if (mine) {
                            float *sb = st + b * SW;
                            if (crit) {   // GRU2 gates of (b, u)
                                const float x = xs[b];
                                const float *Tb = T + b * NT + 3 * U;
                                float gi[3], gh[3];
#pragma unroll
                                for (int g = 0; g < 3; ++g) {
                                    gi[g] = (acc[g] + fmaf(x, S[s.q2 + g * U + u], Tb[g * U + u])) +
                                            S[s.bih2 + g * U + u];
                                    gh[g] = sb[O_GH2 + g * U + u] + S[s.bhh2 + g * U + u];
                                }
                                const float hn = gru_gate_math(gi[0], gi[1], gi[2], gh[0], gh[1], gh[2], sb[O_H2 + u]);
                                sb[O_H2 + u] = hn;
                                put(RH_H2, h2o, b, R, w * U + u, t, hn);
                            } else {      // GH1 of the next step
#pragma unroll
                                for (int g = 0; g < 3; ++g) sb[O_GH1 + g * U + u] = acc[g];
                            }
                        }
                    } else {              // V1h rows r0, r0+1
                        const int jj = jb - nj2, r0 = 2 * (jj % nUF2), bb = jj / nUF2;
                        const int nx = min(kNX, nb - bb * kNX), b = tb0 + bb * kNX + li;
                        float acc[2];
                        fc_block(s.w1, UFv, tl_ + bb * kNX * R, R, nx, r0, acc);
                        if (li < nx) {
                            st[b * SW + O_V1 + r0] = acc[0];
                            if (r0 + 1 < UFv) st[b * SW + O_V1 + r0 + 1] = acc[1];
                        }
                    }
                }
            });
            if (!ok) return;
            signal(RH_H2, t);
            RSTAMP(3);
        }

        // ---- fc1 (:216-218): W1[:, :R]·h2 + V1h + V1c + x·Q3 → f1; with GH2_{t+1} = W_hh2·h2
        RSTAMP(4);
        {
            float *f1o = actp(RH_F1, t);
            const bool ok = run_stage(RH_H2, R, [&](const float *tl_, int tb0, int nb) {
                // [fc1 rows | GH2 of the next step]
                const int nbb = (nb + kNX - 1) / kNX, n1 = nUF2 * nbb, nj1 = round4(n1);
                const int nj2 = nj1 + (SPARSE ? nb : Uv * nbb);
                for (int jb = eng; jb < nj2; jb += kRowsEngines) {
                    if (jb < nj1) {
                        if (jb >= n1) continue;
                        const int r0 = 2 * (jb % nUF2), bb = jb / nUF2;
                        const int nx = min(kNX, nb - bb * kNX), b = tb0 + bb * kNX + li;
                        float acc[2];
                        fc_block(s.w1, UFv, tl_ + bb * kNX * R, R, nx, r0, acc);
                        if (li < nx)
#pragma unroll
                            for (int q = 0; q < 2; ++q) {
                                const int r = r0 + q;
                                if (r >= UFv) break;
                                const float v = acc[q] +
                                                (st[b * SW + O_V1 + r] + fmaf(xs[b], S[s.q3 + r], T[b * NT + 6 * U + r]));
                                put(RH_F1, f1o, b, F, w * UF + r, t, v > 0.0f ? v : 0.0f);
                            }
                    } else {
                        const int jj = jb - nj1;
                        float acc[3];
                        int u, b;
                        bool mine;
                        if (SPARSE) {
                            sparse_gates4(S + s.sp + SP_WHH2 * 3 * s.nbmax * 16, spc + SP_WHH2 * 3 * s.nbmax,
                                          spn + SP_WHH2 * 3, s.nbmax, tl_ + jj * R, li, acc);
                            u = li;
                            b = tb0 + jj;
                            mine = li < Uv;
                        } else {
                            u = jj % Uv;
                            const int bb = jj / Uv, nx = min(kNX, nb - bb * kNX);
                            unit_block(s.whh2, tl_ + bb * kNX * R, R, nx, u, acc);
                            b = tb0 + bb * kNX + li;
                            mine = li < nx;
                        }
                        if (mine)
#pragma unroll
                            for (int g = 0; g < 3; ++g) st[b * SW + O_GH2 + g * U + u] = acc[g];
                    }
                }
            });
            if (!ok) return;
            signal(RH_F1, t);
            RSTAMP(6);
        }

        // ---- fc2 (:220-221): W2[:, :F]·f1 + V2 → f2
        RSTAMP(7);
        {
            float *f2o = actp(RH_F2, t);
            const bool ok = run_stage(RH_F1, F, [&](const float *tl_, int tb0, int nb) {
                const int nbb = (nb + kNX - 1) / kNX, nj = nUF2 * nbb;
                for (int jb = eng; jb < nj; jb += kRowsEngines) {
                    const int r0 = 2 * (jb % nUF2), bb = jb / nUF2;
                    const int nx = min(kNX, nb - bb * kNX), b = tb0 + bb * kNX + li;
                    float acc[2];
                    fc_block(s.w2, UFv, tl_ + bb * kNX * F, F, nx, r0, acc);
                    if (li < nx)
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            const int r = r0 + q;
                            if (r >= UFv) break;
                            const float v = acc[q] + T[b * NT + 6 * U + UF + r];
                            put(RH_F2, f2o, b, F, w * UF + r, t, v > 0.0f ? v : 0.0f);
                        }
                }
            });
            if (!ok) return;
            signal(RH_F2, t);
            RSTAMP(9);
        }

        // ---- fc3 (:223) + sampling (:225-237), distributed by row
        const bool sampler = w < B;
        if (!MOL) {   // fc3 rows are distributed: logits hand-off first
            float *lgo = actp(RH_LG, t);
            const bool ok = run_stage(RH_F2, F, [&](const float *tl_, int tb0, int nb) {
                const int nbb = (nb + kNX - 1) / kNX, nj = nUC2 * nbb;
                for (int jb = eng; jb < nj; jb += kRowsEngines) {
                    const int r0 = 2 * (jb % nUC2), bb = jb / nUC2;
                    const int nx = min(kNX, nb - bb * kNX), b = tb0 + bb * kNX + li;
                    float acc[2];
                    fc_block(s.w3, UCv, tl_ + bb * kNX * F, F, nx, r0, acc);
                    if (li < nx)
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            const int r = r0 + q;
                            if (r >= UCv) break;
                            put(RH_LG, lgo, b, NC, w * UC + r, t, acc[q] + S[s.b3 + r]);
                        }
                }
            });
            if (!ok) return;
            signal(RH_LG, t);
        }
        if (sampler) {
            const int hop = MOL ? RH_F2 : RH_LG;
            const int K = MOL ? F : NC;
            const float *src = actp(hop, t);
            const unsigned long long *gsrc = gran ? a.gact + (size_t)hop * a.gstride : (MOL ? a.gf2 : nullptr);
            if (lead && gsrc) {
                for (int sr = 0; sr < NS && w + sr * G < B; ++sr) {
                    float *dst = tile + sr * ll.KT;
                    auto st_ = [&](int, int j, float v) { dst[j] = v; };
                    gather_chunked<8, 64, decltype(st_)>(gsrc + (size_t)(w + sr * G) * K, K, K, want, a.ctl,
                                                        a.timeout_ticks, t, hop, abort_flag, lane, st_);
                }
            } else if (lead) {
                wait_flags(flagp(hop), G, want, a.ctl, a.timeout_ticks, t, hop, abort_flag);
                if (!*abort_flag)
                    for (int sr = 0; sr < NS && w + sr * G < B; ++sr)
                        dma(tile + sr * ll.KT, src + (size_t)(w + sr * G) * K, K);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            bar();
            RSTAMP(10);
            if (*abort_flag) return;
            if (MOL) {   // the 30 head rows (replicated in every workgroup) against f2 of each sampled row
                if (compute)
                    for (int sr = 0; sr < NS && w + sr * G < B; ++sr)
                        for (int c0 = eng; c0 < NC; c0 += 2 * kRowsEngines) {
                            const int ca = c0, cb = min(c0 + kRowsEngines, NC - 1);
                            const float2 v = row_dot2(head + ca * F, head + cb * F, tile + sr * ll.KT, F / 4, li);
                            if (li == 0) lgs[sr * ll.ncp + ca] = v.x + head[s.b3 - s.w3 + ca];
                            if (li == 0 && c0 + kRowsEngines < NC) lgs[sr * ll.ncp + cb] = v.y + head[s.b3 - s.w3 + cb];
                        }
                bar();
            }
            if (compute)
                for (int sr = wave; sr < NS; sr += kRowsComputeWaves) {
                    const int b = w + sr * G;
                    if (b >= B) break;
                    const float *u = nzs + (t & 1) * NS * ll.nkp + sr * ll.nkp;
                    float x;
                    int label = 0;
                    if (MOL) {
                        x = mol_sample(lgs + sr * ll.ncp, u, lane);
                    } else {
                        label = NC <= 64 * kClsPerLaneMax ? raw_sample<kClsPerLaneMax>(tile + sr * ll.KT, u, NC, lane)
                                                          : raw_sample_any(tile + sr * ll.KT, u, NC, lane);
                        x = label_to_x(label, NC);
                    }
                    if (lane < kXReps) publish(a.xg + (size_t)lane * kXRepStride + b, want, x);
                    if (lane == 0) {
                        const size_t o = (size_t)(a.b0 + b) * a.L + t;
                        a.out[o] = x;
                        if (a.labels) a.labels[o] = label;
                    }
                }
            RSTAMP(11);
        }

        // loader: terms and draws of the next step, while wave 0 collects x
        if (lead && tl + 1 < a.Lc) {
            load_terms(tl + 1, lane, 64);
            load_noise(t + 1, lane, 64);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // ---- x of every row → next step's GRU1
        if (wave == 0)
            gather<kRowsMax / 64, 64>(a.xg + (size_t)(w % kXReps) * kXRepStride, 0, B, B, want, a.ctl,
                                      a.timeout_ticks, t, kRowsHops, abort_flag, lane,
                                      [&](int, int j, float v) { xs[j] = v; });
        bar();
        RSTAMP(12);
        if (*abort_flag) return;
    }

#undef RSTAMP
#undef RSTAMP_T
    // carried state for the next launch of this generate()
    {
        float *cs = a.state + (size_t)w * B * SW;
        for (int i = tid; i < B * SW; i += kRowsThreads) cs[i] = st[i];
        if (w == 0)
            for (int i = tid; i < B; i += kRowsThreads) a.state[(size_t)G * B * SW + i] = xs[i];
    }
}

// --------------------------------------------------------------- conditioning terms input
// X[m][0..KX) for m = tl·B + b:  [cI (R, written by ci_gemm) | a2 a3 a4 (3A) | 1 | 0 0 0]
__global__ void pack_terms_input_kernel(const float *__restrict__ cond, int CD, int Bt, int b0, int B, int t0,
                                        int M, int feat, int A, int R, int KX, float *__restrict__ X) {
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= M) return;
    const int tl = m / B, b = m - tl * B;
    const float *src = cond + ((size_t)(t0 + tl) * Bt + b0 + b) * CD + feat + A;
    float *dst = X + (size_t)m * KX + R;
    for (int k = threadIdx.x & 63; k < KX - R; k += 64) dst[k] = k < 3 * A ? src[k] : (k == 3 * A ? 1.0f : 0.0f);
}

// XCD kernels' terms input: X'[m] = [cond record (CD: mel, a1, a2, a3, a4) | 1 | 0 0 0] — the
// GEMM weights fold I = W_I·[x; mel; a1] + b_I into the W_ih1 / W_ih2 rows (capi.cpp), so no cI.
// split == 0: X' = [cond record | 1 | 0 ...]; split > 0 (the many-row kernel's segmented terms
// GEMM): X'' = [cond[:split] | 1 | cond[split:] | 1 | 0 ...] — a ones column after mel‖a1 and
// another after a4, so the P and V term types each find their bias column inside their K range
// `one`: the value of the ones columns (0 for the frame-rate mel terms, frame_terms.hip)
__global__ void pack_cond_input_kernel(const float *__restrict__ cond, int CD, int Bt, int b0, int B, int t0, int M,
                                       int KX, int split, float one, float *__restrict__ X) {
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= M) return;
    const int tl = m / B, b = m - tl * B;
    const float *src = cond + ((size_t)(t0 + tl) * Bt + b0 + b) * CD;
    float *dst = X + (size_t)m * KX;
    if (split == 0) {
        for (int k = threadIdx.x & 63; k < KX; k += 64) dst[k] = k < CD ? src[k] : (k == CD ? one : 0.0f);
    } else {
        for (int k = threadIdx.x & 63; k < KX; k += 64)
            dst[k] = k < split ? src[k] : k == split ? one : k <= CD ? src[k - 1] : (k == CD + 1 ? one : 0.0f);
    }
}

hipError_t launch_pack_cond_input(const float *cond, int CD, int Bt, int b0, int B, int t0, int Lc, int KX, float *X,
                                  hipStream_t st, int split, float one) {
    const int M = Lc * B;
    hipLaunchKernelGGL(pack_cond_input_kernel, dim3((M + 3) / 4), dim3(256), 0, st, cond, CD, Bt, b0, B, t0, M, KX,
                       split, one, X);
    return hipGetLastError();
}

hipError_t launch_pack_terms_input(const float *cond, int CD, int Bt, int b0, int B, int t0, int Lc, int feat, int A,
                                   int R, int KX, float *X, hipStream_t st) {
    const int M = Lc * B;
    hipLaunchKernelGGL(pack_terms_input_kernel, dim3((M + 3) / 4), dim3(256), 0, st, cond, CD, Bt, b0, B, t0, M, feat,
                       A, R, KX, X);
    return hipGetLastError();
}

// ------------------------------------------------------------------------ host launchers
#define WRNN_ROWS_KERNELS                                                                           \
    (const void *)fatchord_rows_kernel<true, 512, false, false>, (const void *)fatchord_rows_kernel<true, 0, false, false>,   \
        (const void *)fatchord_rows_kernel<false, 512, false, false>,                                           \
        (const void *)fatchord_rows_kernel<false, 0, false, false>, (const void *)fatchord_rows_kernel<true, 0, true, false>,  \
        (const void *)fatchord_rows_kernel<false, 0, true, false>, (const void *)fatchord_rows_kernel<true, 0, false, true>,   \
        (const void *)fatchord_rows_kernel<false, 0, false, true>

static const void *pick_rows_kernel(const RowsArgs &a) {
    const bool sparse = a.s.nbmax > 0;
    const bool d512 = a.R == 512 && a.F == 512 && !sparse;
    if (a.gw) return a.mol ? (const void *)fatchord_rows_kernel<true, 0, false, true>
                           : (const void *)fatchord_rows_kernel<false, 0, false, true>;
    if (a.mol) {
        if (sparse) return (const void *)fatchord_rows_kernel<true, 0, true, false>;
        return d512 ? (const void *)fatchord_rows_kernel<true, 512, false, false>
                    : (const void *)fatchord_rows_kernel<true, 0, false, false>;
    }
    if (sparse) return (const void *)fatchord_rows_kernel<false, 0, true, false>;
    return d512 ? (const void *)fatchord_rows_kernel<false, 512, false, false>
                : (const void *)fatchord_rows_kernel<false, 0, false, false>;
}

// one row group (g1 == nullptr) or two (workgroups [G, 2G) run group 1) in one launch
hipError_t launch_rows(const RowsArgs &a, const RowsGroup *g1, size_t lds_bytes, hipStream_t st) {
    RowsArgs args = a;
    RowsGroup grp = g1 ? *g1 : RowsGroup{};
    int G0 = a.G;
    void *params[] = {&args, &grp, &G0};
    return hipLaunchKernel(pick_rows_kernel(a), dim3(g1 ? 2 * a.G : a.G), dim3(kRowsThreads), params, lds_bytes, st);
}

hipError_t prepare_rows_kernel(int max_lds_bytes) {
    for (const void *k : {WRNN_ROWS_KERNELS}) {
        hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds_bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t rows_occupancy(int *blocks_per_cu, size_t lds_bytes) {
    int best = 1 << 30;
    for (const void *k : {WRNN_ROWS_KERNELS}) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kRowsThreads, lds_bytes);
        if (e != hipSuccess) return e;
        best = n < best ? n : best;
    }
    *blocks_per_cu = best;
    return hipSuccess;
}

}  // namespace wrnn
