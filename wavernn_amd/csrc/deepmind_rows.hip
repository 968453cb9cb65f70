// deepmind_rows.hip — persistent CDNA4 kernel for the dual coarse/fine softmax WaveRNN
// (models/deepmind_version.py:75-165, BASELINE config 5) over B independent rows (utterances).
//
// Per step (reference order, :101-156):
//   coarse gates from R·h_{t-1} (own rows) + I_coarse·[c_{t-1}, f_{t-1}] → h_c   → [hc]
//   O1·h_c → relu                                                                → [o1]
//   O2 → coarse logits                                                           → [lc]
//   sample c_t (row-distributed, argmax(p/q))                                    → [x: c_t]
//   fine gates from R·h_{t-1} (own rows) + I_fine·[c_{t-1}, f_{t-1}, c_t] → h_f  → [hf]
//   O3·h_f → relu                                                                → [o3]
//   O4 → fine logits                                                             → [lf]
//   sample f_t                                                                   → [x: f_t]
// R·h_t for the next step is accumulated off the critical path in two halves: the columns
// on h_c while O1 runs (hc tiles), the columns on h_f while O3 runs (hf tiles), into a
// parity-double-buffered per-row state.  Hand-offs and engines are those of fatchord_rows.hip
// (rows_device.h): bulk sc1 stores → flag, loader-wave DMA of row tiles, register-blocked
// 16-lane dots; the sampled labels travel as tagged granules.
// Arithmetic: fp32; the coarse/fine labels are the bit-exact quantity.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "deepmind_rows.h"
#include "rows_device.h"

namespace wrnn {

// kS = 448 instantiates the shipped dims (hidden 896) with compile-time dot lengths.
// Row groups as in fatchord_rows.hip: workgroups [G0, 2·G0) run a second, independent instance
// over the rows of g1 (half the flags per hop, half the rows streamed per stage).
// GW: the slab stays in HBM (hidden sizes whose weights exceed LDS), as fatchord_rows.hip's GW.
template <int kS, bool GW>
__global__ __launch_bounds__(kDmThreads) void deepmind_rows_kernel(DmArgs a, DmGroup g1, int G0) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, row = lane >> 4;
    const bool grp1 = (int)blockIdx.x >= G0;
    if (grp1) {
        a.act = g1.act;
        a.flags = g1.flags;
        a.xg = g1.xg;
        a.gact = g1.gact;
        a.state = g1.state;
        a.row0 = g1.row0;
        a.B = g1.B;
        a.b0 = g1.b0;
    }
    const int w = (int)blockIdx.x - (grp1 ? G0 : 0);
    const int S = kS ? kS : a.S, H = 2 * S, Q = a.Q, U = a.U, UO = a.UO, UO2 = a.UO2, G = a.G, B = a.B;
    const int TB = a.TB, KA = a.KA;
    const DmLds ll = dm_lds_layout(GW ? 0 : a.s.total, B, TB, S, Q, U, G);
    const DmSlab &s = a.s;
    const float *W = GW ? a.slab + (size_t)w * s.total : smem + ll.slab;
    float *tile = smem + ll.tile, *st = smem + ll.st, *pcv = smem + ll.pc, *pfv = smem + ll.pf;
    float *nzs = smem + ll.nz;
    int *abort_flag = reinterpret_cast<int *>(smem + ll.flag);
    float *ccur = smem + ll.cs, *cnew = smem + ll.cn;
    const int SW = ll.SW, NS = ll.NS;
    const int O_HF = U, O_RH = 2 * U;
    auto RH = [&](int par, int half, int k6, int u) { return O_RH + ((((par & 1) * 2 + half) * 6 + k6) * U + u); };
    const int Uv = max(0, min(U, S - w * U));
    const int UOv = max(0, min(UO, S - w * UO));
    const int UO2v = max(0, min(UO2, Q - w * UO2));
    const bool loader = wave >= kLoaderWave;           // waves 4-7: tile DMA (split four ways)
    const bool lead = wave == kLoaderWave;             // wave 4: flag polls, draws, samplers
    const bool compute = !loader;
    int *go = abort_flag + 1;                          // LDS: wave 4 → the other loaders, "flags seen"
    const int eng = wave * 4 + row;
    const size_t hop_sz = (size_t)2 * B * KA;
    auto actp = [&](int hop, int t) { return a.act + hop * hop_sz + (size_t)(t & 1) * B * KA; };
    auto flagp = [&](int hop) { return a.flags + (size_t)hop * kFlagSlots * kFlagStride; };
    const bool gran = a.gact != nullptr;
    auto signal = [&](int hop, int t) {
        if (!gran && tid == 0)
            __hip_atomic_store(flagp(hop) + w * kFlagStride, (unsigned)t + 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };
    // one activation value (row b, column k, row stride K) of hop `hop` at step t: a granule, or
    // an sc1 store into the bulk matrix
    auto put = [&](int hop, float *bulk, int b, int K, int k, int t, float v) {
        if (gran) publish(a.gact + (size_t)hop * a.gstride + (size_t)b * K + k, (uint32_t)t + 1u, v);
        else store_sc1(bulk + (size_t)b * K + k, v);
    };
    // granule mode: rows [r0, r0 + nr) of a hop polled by the four loader waves into LDS (stride K)
    auto gran_tile = [&](float *dst, int hop, int K, int r0, int nr, int t) {
        const int lid = (wave - kLoaderWave) * 64 + lane;
        auto st_ = [&](int b, int j, float v) { dst[b * K + j] = v; };
        gather_chunked<kDmGranNG, 64 * kDmLoaders, decltype(st_)>(
            a.gact + (size_t)hop * a.gstride + (size_t)r0 * K, nr * K, K, (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t,
            hop, abort_flag, lid, st_);
    };
    auto gran_tile_all = [&](float *dst, int hop, int K, int r0, int nr, int t) {   // every wave
        auto st_ = [&](int b, int j, float v) { dst[b * K + j] = v; };
        gather_chunked<kDmGranNG, kDmThreads, decltype(st_)>(
            a.gact + (size_t)hop * a.gstride + (size_t)r0 * K, nr * K, K, (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t,
            hop, abort_flag, tid, st_);
    };
    auto xgp = [&](int which) { return a.xg + (size_t)which * kXReps * kXRepStride; };
    auto dma = [&](float *dst, const float *src, int n) {
        for (int c = 0; c < n; c += 256)
            if (c + lane * 4 < n)
                __builtin_amdgcn_global_load_lds(WRNN_GPTR(src + c + lane * 4), WRNN_LPTR(dst + c), 16, 0, 16);
    };
    // the same split over the four loader waves (1 KiB pieces, round robin): one wave streams a
    // fresh tile at only ~15 GB/s (MI355X_MICROARCH.md handoff-payload)
    auto dma_part = [&](float *dst, const float *src, int n) {
        for (int c = (wave - kLoaderWave) * 256; c < n; c += kDmLoaders * 256)
            if (c + lane * 4 < n)
                __builtin_amdgcn_global_load_lds(WRNN_GPTR(src + c + lane * 4), WRNN_LPTR(dst + c), 16, 0, 16);
    };
    // draws of step t for the sampled rows: [q_coarse (Q) | q_fine (Q)], Exp(1)
    auto load_noise = [&](int t, int id, int nl) {
        float *slot = nzs + (t & 1) * NS * ll.nkp;
        for (int i = id; i < NS * 2 * Q; i += nl) {
            const int sr = i / (2 * Q), k = i - sr * 2 * Q, b = w + sr * G;
            if (b >= B) continue;
            slot[sr * ll.nkp + k] = a.noise ? a.noise[((size_t)t * a.Bt + a.b0 + b) * 2 * Q + k]
                                            : philox_noise(a.seed, (unsigned long long)(a.row0 + b), (uint32_t)t,
                                                           (uint32_t)k, 0);
        }
    };

    // ---- prologue: weights, carried state (h, R·h partials, previous labels), first draws
    {
        const float4 *src = reinterpret_cast<const float4 *>(a.slab + (size_t)w * s.total);
        float4 *dst = reinterpret_cast<float4 *>(smem + ll.slab);
        if (!GW)
            for (int i = tid; i < s.total / 4; i += kDmThreads) dst[i] = src[i];
        const float *cs = a.state + (size_t)w * B * SW;
        for (int i = tid; i < B * SW; i += kDmThreads) st[i] = a.t0 > 0 ? cs[i] : 0.0f;
        const float *cx = a.state + (size_t)G * B * SW;
        for (int i = tid; i < B; i += kDmThreads) {   // out_coarse = out_fine = 0 initially (:89-90)
            pcv[i] = a.t0 > 0 ? cx[i] : 0.0f;
            pfv[i] = a.t0 > 0 ? cx[B + i] : 0.0f;
        }
        if (tid == 0) {
            *abort_flag = 0;
            *go = -1;
        }
        load_noise(a.t0, tid, kDmThreads);
    }
    __syncthreads();

    constexpr int kNX = 4;
    constexpr int KI = kS / 64;
    auto tbuf = [&](int k) { return tile + (k & 1) * TB * ll.KT; };
    int t_cur = a.t0;
    auto run_stage = [&](int hop, int K, auto &&jobs) -> bool {
        const float *src = actp(hop, t_cur);
        const int ntiles = (B + TB - 1) / TB;
        if (gran) {
            gran_tile_all(tbuf(0), hop, K, 0, min(TB, B), t_cur);
        } else if (loader) {   // wave 4 polls the flags and releases waves 5-7 through an LDS word
            const int go_val = (t_cur + 1) * kDmHops + hop;
            if (lead) {
                wait_flags(flagp(hop), G, (unsigned)t_cur + 1u, a.ctl, a.timeout_ticks, t_cur, hop, abort_flag);
                __hip_atomic_store(go, go_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                while (__hip_atomic_load(go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != go_val)
                    __builtin_amdgcn_s_sleep(1);
            }
            if (!*reinterpret_cast<volatile int *>(abort_flag)) dma_part(tbuf(0), src, min(TB, B) * K);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        if (*abort_flag) return false;
        for (int k = 0; k < ntiles; ++k) {
            const int tb0 = k * TB, nb = min(TB, B - tb0);
            if (loader && k + 1 < ntiles) {
                if (gran) {
                    gran_tile(tbuf(k + 1), hop, K, tb0 + TB, min(TB, B - tb0 - TB), t_cur);
                } else {
                    dma_part(tbuf(k + 1), src + (size_t)(tb0 + TB) * K, min(TB, B - tb0 - TB) * K);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            if (compute) jobs(tbuf(k), tb0, nb);
            bar();
        }
        if (!gran) {   // bulk: every storing wave drains before the stage's signal
            if (compute) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
        }
        return true;
    };
    // output rows r0, r0+1 of an S-input layer (O1..O4) on 4 activation rows
    auto out_block = [&](int wbase, int nrows, const float *x, int nx, int r0, float (&acc)[2]) {
        const int r1 = r0 + 1 < nrows ? r0 + 1 : r0;
        bdot4<2, KI>(W + wbase + r0 * S, (r1 - r0) * S, x, S, nx, S / 4, li, acc);
    };
    // the 3 gate rows (u, r, e) of own unit u of half h2 (0 coarse, 1 fine), columns [c0, c0 + S)
    auto r_block = [&](int h2, int u, int c0, const float *x, int nx, float (&acc)[3]) {
        bdot4<3, KI>(W + s.rw + (size_t)((h2 * 3) * U + u) * H + c0, U * H, x, S, nx, S / 4, li, acc);
    };
    const int nUO = (UOv + 1) / 2, nUO2 = (UO2v + 1) / 2;
    // a layer stage: [out rows → act (relu optional) | R half-columns of the next step]
    auto layer_jobs = [&](int wbase, int bbase, int nrows, int nstep, bool relu, int dhop, float *dst, int dstK,
                          int rowoff, int rhalf, int next_par, int t) {
        return [=, &st, &put](const float *tl_, int tb0, int nb) {
            const int nbb = (nb + kNX - 1) / kNX, n1 = nstep * nbb, nj1 = round4(n1);
            const int nj2 = nj1 + (rhalf >= 0 ? 2 * Uv * nbb : 0);
            for (int jb = eng; jb < nj2; jb += kDotEngines) {
                if (jb < nj1) {
                    if (jb >= n1) continue;
                    const int r0 = 2 * (jb % nstep), bb = jb / nstep;
                    const int nx = min(kNX, nb - bb * kNX), b = tb0 + bb * kNX + li;
                    float acc[2];
                    out_block(wbase, nrows, tl_ + bb * kNX * S, nx, r0, acc);
                    if (li < nx)
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            const int r = r0 + q;
                            if (r >= nrows) break;
                            float v = acc[q] + W[bbase + r];
                            if (relu) v = v > 0.0f ? v : 0.0f;
                            put(dhop, dst, b, dstK, rowoff + r, t, v);
                        }
                } else {
                    const int jj = jb - nj1, hu = jj % (2 * Uv), bb = jj / (2 * Uv);
                    const int h2 = hu / Uv, u = hu - h2 * Uv;
                    const int nx = min(kNX, nb - bb * kNX), b = tb0 + bb * kNX + li;
                    float acc[3];
                    r_block(h2, u, rhalf * S, tl_ + bb * kNX * S, nx, acc);
                    if (li < nx)
#pragma unroll
                        for (int g = 0; g < 3; ++g) st[b * SW + RH(next_par, rhalf, h2 * 3 + g, u)] = acc[g];
                }
            }
        };
    };
    // gate update of own units of half h2 for every row; x3 = third I_fine input (fine only)
    auto gates = [&](int h2, int par, int dhop, float *dst, const float *xcur, int t) {
        for (int i = tid; i < B * Uv; i += kCompute) {
            const int b = i / Uv, u = i - b * Uv, j = w * U + u;
            const float x0 = label_x(pcv[b]), x1 = label_x(pfv[b]);   // (:106-108)
            float *sb = st + b * SW;
            float I[3];
#pragma unroll
            for (int g = 0; g < 3; ++g) {   // I_coarse / I_fine rows: separately rounded products (:111, :137)
                if (h2 == 0) {
                    const float *wi = W + s.ic + (g * U + u) * 2;
                    I[g] = __fadd_rn(__fmul_rn(wi[0], x0), __fmul_rn(wi[1], x1));
                } else {
                    const float *wi = W + s.if_ + (g * U + u) * 3;
                    const float x2 = label_x(xcur[b]);                                    // (:135-136)
                    I[g] = __fadd_rn(__fadd_rn(__fmul_rn(wi[0], x0), __fmul_rn(wi[1], x1)), __fmul_rn(wi[2], x2));
                }
            }
            float Rg[3];
#pragma unroll
            for (int g = 0; g < 3; ++g) Rg[g] = sb[RH(par, 0, h2 * 3 + g, u)] + sb[RH(par, 1, h2 * 3 + g, u)];
            // (:122-125 / :142-145)
            const float uu = sigmoid_((Rg[0] + I[0]) + W[s.bu + h2 * U + u]);
            const float rr = sigmoid_((Rg[1] + I[1]) + W[s.br + h2 * U + u]);
            const float ee = tanh_((rr * Rg[2] + I[2]) + W[s.be + h2 * U + u]);
            const float hn = uu * sb[h2 * O_HF + u] + (1.0f - uu) * ee;
            sb[h2 * O_HF + u] = hn;
            put(dhop, dst, b, S, j, t, hn);
        }
    };
    // row-distributed sampling from the logits hop; publishes the label granule
    auto sample = [&](int hop, int which, int t, bool fine) -> bool {
        if (w >= B) return true;
        const float *src = actp(hop, t);
        if (lead && gran) {
            for (int sr = 0; sr < NS && w + sr * G < B; ++sr) {
                float *dst = tile + sr * ll.KT;
                auto st_ = [&](int, int j, float v) { dst[j] = v; };
                gather_chunked<8, 64, decltype(st_)>(a.gact + (size_t)hop * a.gstride + (size_t)(w + sr * G) * Q, Q, Q,
                                                    (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t, hop, abort_flag, lane,
                                                    st_);
            }
        } else if (lead) {
            wait_flags(flagp(hop), G, (unsigned)t + 1u, a.ctl, a.timeout_ticks, t, hop, abort_flag);
            if (!*abort_flag)
                for (int sr = 0; sr < NS && w + sr * G < B; ++sr) dma(tile + sr * ll.KT, src + (size_t)(w + sr * G) * Q, Q);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        if (*abort_flag) return false;
        if (compute)
            for (int sr = wave; sr < NS; sr += kWaves) {
                const int b = w + sr * G;
                if (b >= B) break;
                const float *q = nzs + (t & 1) * NS * ll.nkp + sr * ll.nkp + (fine ? Q : 0);
                const int label = Q <= 256 ? raw_sample<4>(tile + sr * ll.KT, q, Q, lane)
                                           : raw_sample_any(tile + sr * ll.KT, q, Q, lane);
                if (lane < kXReps) publish(xgp(which) + (size_t)lane * kXRepStride + b, (uint32_t)t + 1u, (float)label);
                if (!fine) {
                    if (lane == 0) ccur[sr] = (float)label;
                } else if (lane == 0) {
                    const int v = (int)ccur[sr] * 256 + label - 32768;     // combine_signal, utils/dsp.py:33
                    const size_t o = (size_t)(a.b0 + b) * a.L + t;
                    a.out[o] = (float)v;
                    if (a.labels) a.labels[o] = v;
                }
            }
        return true;
    };
    auto gather_labels = [&](int which, int t, float *dst) {
        if (wave == 0)
            gather<kRowsMax / 64, 64>(xgp(which) + (size_t)(w % kXReps) * kXRepStride, 0, B, B, (uint32_t)t + 1u,
                                      a.ctl, a.timeout_ticks, t, kDmHops + which, abort_flag, lane,
                                      [&](int, int j, float v) { dst[j] = v; });
    };

    for (int tl = 0; tl < a.Lc; ++tl) {
        const int t = a.t0 + tl, par = t & 1;
        t_cur = t;
        // ---- coarse gates → h_c
        if (compute) {
            gates(0, par, DH_HC, actp(DH_HC, t), nullptr, t);
            if (!gran) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        signal(DH_HC, t);
        // ---- O1 (relu) on h_c; R[:, :S]·h_c for the next step
        if (!run_stage(DH_HC, S, layer_jobs(s.o1, s.o1b, UOv, nUO, true, DH_O1, actp(DH_O1, t), S, w * UO, 0, t + 1, t))) return;
        signal(DH_O1, t);
        // ---- O2 → coarse logits
        if (!run_stage(DH_O1, S, layer_jobs(s.o2, s.o2b, UO2v, nUO2, false, DH_LC, actp(DH_LC, t), Q, w * UO2, -1, 0, t))) return;
        signal(DH_LC, t);
        // ---- sample c_t; everyone collects c_t of every row
        if (!sample(DH_LC, 0, t, false)) return;
        gather_labels(0, t, cnew);
        bar();
        if (*abort_flag) return;
        // ---- fine gates → h_f
        if (compute) {
            gates(1, par, DH_HF, actp(DH_HF, t), cnew, t);
            if (!gran) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        signal(DH_HF, t);
        // ---- O3 (relu) on h_f; R[:, S:]·h_f for the next step
        if (!run_stage(DH_HF, S, layer_jobs(s.o3, s.o3b, UOv, nUO, true, DH_O3, actp(DH_O3, t), S, w * UO, 1, t + 1, t))) return;
        signal(DH_O3, t);
        // ---- O4 → fine logits
        if (!run_stage(DH_O3, S, layer_jobs(s.o4, s.o4b, UO2v, nUO2, false, DH_LF, actp(DH_LF, t), Q, w * UO2, -1, 0, t))) return;
        signal(DH_LF, t);
        // ---- sample f_t; collect f_t of every row; previous labels ← (c_t, f_t)
        if (!sample(DH_LF, 1, t, true)) return;
        if (lead && tl + 1 < a.Lc) {
            load_noise(t + 1, lane, 64);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        gather_labels(1, t, pfv);
        for (int i = tid; i < B; i += kDmThreads) pcv[i] = cnew[i];
        bar();
        if (*abort_flag) return;
    }

    {
        float *cs = a.state + (size_t)w * B * SW;
        for (int i = tid; i < B * SW; i += kDmThreads) cs[i] = st[i];
        if (w == 0)
            for (int i = tid; i < B; i += kDmThreads) {
                a.state[(size_t)G * B * SW + i] = pcv[i];
                a.state[(size_t)G * B * SW + B + i] = pfv[i];
            }
    }
}

#define WRNN_DM_KERNELS                                                                              \
    (const void *)deepmind_rows_kernel<448, false>, (const void *)deepmind_rows_kernel<0, false>,      \
        (const void *)deepmind_rows_kernel<0, true>

static const void *pick_dm_kernel(const DmArgs &a) {
    if (a.gw) return (const void *)deepmind_rows_kernel<0, true>;
    return a.S == 448 ? (const void *)deepmind_rows_kernel<448, false> : (const void *)deepmind_rows_kernel<0, false>;
}

hipError_t launch_dm(const DmArgs &a, const DmGroup *g1, size_t lds_bytes, hipStream_t st) {
    DmArgs args = a;
    DmGroup grp = g1 ? *g1 : DmGroup{};
    int G0 = a.G;
    void *params[] = {&args, &grp, &G0};
    return hipLaunchKernel(pick_dm_kernel(a), dim3(g1 ? 2 * a.G : a.G), dim3(kDmThreads), params, lds_bytes, st);
}

hipError_t prepare_dm_kernel(int max_lds_bytes) {
    for (const void *k : {WRNN_DM_KERNELS}) {
        hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds_bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t dm_occupancy(int *blocks_per_cu, size_t lds_bytes) {
    int best = 1 << 30;
    for (const void *k : {WRNN_DM_KERNELS}) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kDmThreads, lds_bytes);
        if (e != hipSuccess) return e;
        best = n < best ? n : best;
    }
    *blocks_per_cu = best;
    return hipSuccess;
}

}  // namespace wrnn
