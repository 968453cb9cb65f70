// fatchord_split.hip — role-split persistent kernel for ONE MoL row (the batch-1 headline).
//
// Same loop as fatchord_loop.hip (models/fatchord_version.py:201-241), but the workgroups take
// two roles so that every critical hand-off has few participants (a hop's cost grows with the
// number of producers and pollers: 2 → 0.47 µs, 32 → 1.0, 256 → 1.7 µs, tools/hopbench.hip):
//
//   GRU workgroups (Gg = R/4): 4 hidden units of both GRUs.  GRU1 runs for ALL units in every
//     GRU workgroup (local gate math on gathered terms, as in fatchord_loop.hip), GRU2 for the
//     own units; each publishes y_j = x_I,j + h1_j + h2_j (fc1's input, :212-216) and h2_j.
//   FC workgroups (Gf = F/16): 16 rows of fc1 and of fc2, one per 16-lane engine, and the fc3
//     columns of its f2 rows: it publishes 30 partial logits W3[:, own rows]·f2[own rows].
//   Every GRU workgroup gathers the partial logits, sums them and runs the MoL sampler
//     redundantly (bit-identical), so the sample needs no hand-off of its own; the FC
//     workgroups need no x.
//
// Critical path per step:
//   x_{t-1} → GRU1 (all units) → W_ih2[:, :R]·h1 → GRU2 gates → [hop Y: Gg → Gf]
//   → W1[:, :R]·y → [hop F1: Gf → Gf] → W2[:, :F]·f1 → fc3 partials → [hop F2: Gf → Gg]
//   → Σ partials + b3 → sample → x_t
// Off the critical path, while fc1/fc2 run in the FC workgroups, the GRU workgroups compute
// GH1 = W_hh1·h1_t → publish step t+1's GRU1 terms, gather h2_t → GH2 = W_hh2·h2_t, and
// gather step t+1's terms of all units.  Everything that depends only on the conditioning
// (P1 = W_ih1·cI, P2 = W_ih2·[cI; a2], V1c = W1[:, R:]·a3 + b1, V2 = W2[:, F:]·a4 + b2, and
// cI itself) comes from one fp32 GEMM before the launch (capi.cpp) and is streamed into an LDS
// ring by the loader wave, so the LDS holds only the loop matrices (and, FC, 16 fc3 columns).
//
// Arithmetic is fp32; the sums are re-associated like fatchord_loop.hip's (tolerance-checked
// against the oracle).  Every wait is bounded; a timeout sets the abort word.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fatchord_split.h"
#include "wrnn_device.h"

namespace wrnn {

#ifndef WRNN_OFF_SLEEP
#define WRNN_OFF_SLEEP 32
#endif
constexpr int kOffSleep = WRNN_OFF_SLEEP;   // backoff (×64 cycles) of the off-critical polls
static_assert(kOffSleep >= 0 && kOffSleep <= 127, "s_sleep takes a 7-bit count");
// (same-box sweep, MI355X, us/step: 2 → 5.97, 12 → 5.89, 24 → 5.89, 32 → 5.83, 48 → 5.85;
// fewer polls of the off-critical vectors leave the L2 channels to the critical hand-offs)
#ifndef WRNN_DRAIN_PUB
#define WRNN_DRAIN_PUB 1
#endif
constexpr bool kDrainPub = WRNN_DRAIN_PUB;
#ifndef WRNN_SPLIT_PK
#define WRNN_SPLIT_PK 1
#endif
constexpr bool kPk = WRNN_SPLIT_PK;          // critical dots as packed FMAs in 4 chains (row_dot_pk)
#ifndef WRNN_SPLIT_PRE
#define WRNN_SPLIT_PRE 1
#endif
constexpr bool kPre = WRNN_SPLIT_PRE;        // operands of the post-dot math read from LDS ahead

// a critical-path 16-lane row dot over K floats
template <int K>
__device__ __forceinline__ float crit_dot(const float *__restrict__ w, const float *__restrict__ x, int li) {
    if constexpr (kPk) return row_dot_pk<K / 4>(w, x, li);
    else return row_dot(w, x, K / 4, li);
}

#define SSTAMP(k)                                                                                          \
    do {                                                                                                   \
        if (dbg_on && tid == 0) stamp[(t & 1) * kStamps + (k)] = (unsigned)__builtin_amdgcn_s_memrealtime(); \
    } while (0)

// kDbg: the WRNN_DEBUG_STAMPS build of the kernel (stamp code compiled out of the production one)
template <int kR, int kF, bool kDbg>
__global__ __launch_bounds__(kThreads) void fatchord_split_kernel(SplitArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int R = kR, F = kF, NC = 30, RT = kTermsPerUnit * R;
    constexpr int NG_R = R / kPollThreads, NG_F = F / kPollThreads;
    static_assert(R % kPollThreads == 0 && F % kPollThreads == 0 && NG_R <= 16 && NG_F <= 16, "poll layout");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, row = lane >> 4;
    const int w = blockIdx.x;
    const bool gru = w < a.Gg;
    const int g = gru ? w : w - a.Gg;                 // index within the role
    const SplitLds ll = split_lds_layout(a.gs.total > a.fs.total ? a.gs.total : a.fs.total, R, F);
    const float *S = smem + ll.slab;
    float *va = smem + ll.va, *vb = smem + ll.vb, *f2 = smem + ll.f2, *sg = smem + ll.sg;
    float *ring = smem + ll.ring, *nzr = smem + ll.nz, *gh2 = smem + ll.gh2, *gh1 = smem + ll.gh1;
    float *h2own = smem + ll.h2own, *xprev = smem + ll.xprev;
    int *abort_flag = reinterpret_cast<int *>(smem + ll.flag);
    unsigned *stamp = reinterpret_cast<unsigned *>(smem + ll.stamp);
    const bool loader = wave == kLoaderWave;
    const bool dbg_on = kDbg && a.dbg != nullptr;
    const int N = (a.Gg + a.Gf) * kSplitTerms;        // terms per step, all workgroups
    const int term0 = w * kSplitTerms;                // this workgroup's columns
    const int t_end = a.t0 + a.Lc;
    const int t_terms = min(t_end, a.L - 1);          // last step with a terms row in this launch
    const size_t hop_stride = (size_t)a.reps * a.rep_stride;
    const size_t poll_off = (size_t)(w % a.reps) * a.rep_stride;
    auto XG = [&](int hop) { return a.xg + (size_t)hop * hop_stride; };
    auto RING = [&](int t) { return ring + (t & (kSplitRing - 1)) * kSplitTerms; };
    auto NZ = [&](int t) { return nzr + (t & (kSplitRing - 1)) * kSplitNoise; };

    // the sampler's 11 noise terms of step t (lanes 0..10 of one wave): u1 → log(-log u1)
    // (distribution.py:107), u2 → log u2 − log(1 − u2) (:119), prepared ahead of time
    auto fill_noise = [&](int t) {
        if (lane < 11) {
            float uu;
            if (a.noise) uu = a.noise[((size_t)t * a.Bt + a.b0) * 11 + lane];
            else uu = philox_noise(a.seed, (unsigned long long)a.row0, (uint32_t)t, (uint32_t)lane, 1);
            NZ(t)[lane] = mol_noise_term(uu, lane);
        }
    };
    // GRU1 terms of step t for the own units → every replica of the S(t) vector (one wave):
    //   S_r = (GH1_r + b_hh,r) + (P1_r + b_ih,r), S_z likewise, Gi_n = P1_n + b_ih,n, Gh_n = GH1_n + b_hh,n
    auto publish_terms = [&](int t, bool zero_gh) {
        const float *p1 = RING(t) + ST_P1;
        for (int idx = lane; idx < kSplitUnits * kTermsPerUnit * a.reps; idx += 64) {
            const int k16 = idx / a.reps, rep = idx - k16 * a.reps;
            const int u = k16 >> 2, term = k16 & 3;
            const float *bh = S + a.gs.bhh1 + u * 3, *bi = S + a.gs.bih1 + u * 3;
            const float g_r = zero_gh ? 0.0f : gh1[u * 3 + 0];
            const float g_z = zero_gh ? 0.0f : gh1[u * 3 + 1];
            const float g_n = zero_gh ? 0.0f : gh1[u * 3 + 2];
            float v;
            if (term == 0) v = (g_r + bh[0]) + (p1[u * 3 + 0] + bi[0]);
            else if (term == 1) v = (g_z + bh[1]) + (p1[u * 3 + 1] + bi[1]);
            else if (term == 2) v = p1[u * 3 + 2] + bi[2];
            else v = g_n + bh[2];
            publish(XG(SH_S0 + (t & 1)) + (size_t)rep * a.rep_stride + (size_t)(g * kSplitUnits + u) * kTermsPerUnit + term,
                    (uint32_t)t + 1u, v);
        }
    };
    auto store_sg = [&](int, int j, float v) { sg[j] = v; };
    auto gather_terms = [&](int t) {   // off the critical path: polls back off (kOffSleep)
        gather_chunked<NG_R, kPollThreads, decltype(store_sg), kOffSleep>(
            XG(SH_S0 + (t & 1)) + poll_off, RT, RT, (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t, SH_S0 + (t & 1),
            abort_flag, lane, store_sg);
    };
    // fc3 logits of step t (:223) from the FC workgroups' partial sums (hop F2), one wave: lane l
    // polls logit j = l & 31 of producers (l >> 5)·kPh … +kPh-1 and sums them pairwise; the two
    // halves meet across the wave (identical bits in both), + b3.  Lanes with j >= 30 re-read
    // logit 0 (their result is not used).
    constexpr int kPh = F / kSplitFcRows / 2;
    static_assert(kPh >= 1 && (kPh & (kPh - 1)) == 0 && kPh <= 16, "logit gather layout");
    auto gather_logits = [&](uint32_t tag, int t) -> float {
        const int j = lane & 31, jj = j < NC ? j : 0;
        const float b3 = S[a.gs.b3 + jj];
        const unsigned long long *gp = XG(SH_F2) + poll_off + (size_t)(lane >> 5) * kPh * kSplitLogitLine + jj;
        const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
        unsigned spins = 0;
        float p[kPh];
        for (;;) {
            unsigned long long v[kPh];
#pragma unroll
            for (int k = 0; k < kPh; ++k)
                v[k] = __hip_atomic_load(gp + k * kSplitLogitLine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool ok = true;
#pragma unroll
            for (int k = 0; k < kPh; ++k) ok &= (uint32_t)(v[k] >> 32) == tag;
            if (ok) {
#pragma unroll
                for (int k = 0; k < kPh; ++k) p[k] = __uint_as_float((uint32_t)v[k]);
                break;
            }
            if ((++spins & 63u) == 0) {
                const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (late || other) {
                    if (late) record_abort(a.ctl, -4, t, SH_F2, w);
                    *abort_flag = 1;
#pragma unroll
                    for (int k = 0; k < kPh; ++k) p[k] = 0.0f;
                    break;
                }
            }
        }
#pragma unroll
        for (int n = kPh / 2; n >= 1; n /= 2)
#pragma unroll
            for (int k = 0; k < n; ++k) p[k] += p[k + n];
        float s = p[0];
        s += __shfl_xor(s, 32);
        return s + b3;
    };

    // ---- prologue: slab → LDS, state (zero, or carried from the previous time chunk), the
    // terms and noise of the first two steps; at t = 0 the GRU1 terms of step 0 (GH1 = 0)
    {
        const float *src = gru ? a.gslab + (size_t)g * a.gs.total : a.fslab + (size_t)g * a.fs.total;
        const int n4 = (gru ? a.gs.total : a.fs.total) / 4;
        for (int i = tid; i < n4; i += kThreads)
            reinterpret_cast<float4 *>(smem + ll.slab)[i] = reinterpret_cast<const float4 *>(src)[i];
        const bool resume = a.t0 > 0 && gru;
        const float *st = a.state + (size_t)w * split_state_w(R);
        for (int i = tid; i < R; i += kThreads) {
            va[i] = resume ? st[i] : 0.0f;
            vb[i] = resume ? st[R + i] : 0.0f;
        }
        if (gru)
            for (int i = tid; i < RT; i += kThreads) sg[i] = resume ? st[2 * R + i] : 0.0f;
        if (tid < 24) gh2[tid] = resume ? st[6 * R + tid] : 0.0f;
        if (tid < 4) {
            h2own[tid] = resume ? st[6 * R + 24 + tid] : 0.0f;
            abort_flag[tid] = 0;
        }
        if (tid == 0) xprev[(a.t0 + 1) & 1] = a.t0 > 0 ? a.state[(size_t)w * split_state_w(R) + 6 * R + 28] : 0.0f;
        for (int t = a.t0; t < a.t0 + 2; ++t) {
            if (t <= t_terms)
                for (int i = tid; i < kSplitTerms; i += kThreads)
                    RING(t)[i] = a.terms[(size_t)(t - a.t0) * N + term0 + i];
            if (wave == 1 && t < a.L) fill_noise(t);
        }
    }
    __syncthreads();
    if (gru && a.t0 == 0) {
        if (wave == 1) publish_terms(0, true);
        if (wave == 3) gather_terms(0);
    }
    __syncthreads();
    if (*abort_flag) return;

    // loader wave, after the first barrier of step t: the output of step t-1, the noise of
    // step t+2 and its terms (LDS-DMA, waited for before the step's last barrier)
    auto loader_top = [&](int t) {
        if (dbg_on && t > a.t0 && t - 1 - a.t0 < a.dbg_steps && lane < kStamps)
            a.dbg[((size_t)w * a.dbg_steps + (t - 1 - a.t0)) * kStamps + lane] = stamp[((t - 1) & 1) * kStamps + lane];
        if (w == 0 && lane == 0 && t > a.t0) a.out[(size_t)a.b0 * a.L + (t - 1)] = xprev[(t - 1) & 1];
        const int t2 = t + 2;
        if (t2 < a.L) fill_noise(t2);
        if (t2 <= t_terms && lane < kSplitTerms / 4)
            __builtin_amdgcn_global_load_lds(WRNN_GPTR(a.terms + (size_t)(t2 - a.t0) * N + term0 + lane * 4),
                                             WRNN_LPTR(RING(t2)), 16, 0, 0);
    };

    float x = xprev[(a.t0 + 1) & 1];   // x_{t-1}, wave-uniform in every compute wave
    for (int t = a.t0; t < t_end; ++t) {
        const uint32_t tag = (uint32_t)t + 1u;
        const bool more = t + 1 < a.L;
        SSTAMP(0);
        if (gru) {
            // GRU2's per-unit operands (all known before x): issued now, landed during GRU1
            float pq2[3], pp2[3], pbi[3], pgh[3], pwi0 = 0.0f, pci = 0.0f, ph2 = 0.0f;
            if (kPre && !loader) {
                const int u = wave;
                const float *tr = RING(t);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    pq2[q] = S[a.gs.q2 + u * 3 + q];
                    pp2[q] = tr[ST_P2 + u * 3 + q];
                    pbi[q] = S[a.gs.bih2 + u * 3 + q];
                    pgh[q] = gh2[(t & 1) * 12 + u * 3 + q] + S[a.gs.bhh2 + u * 3 + q];
                }
                pwi0 = S[a.gs.wi0 + u];
                pci = tr[ST_CI + u];
                ph2 = h2own[u];
            }
            // ---- A: GRU1 (:208-210) for all units from the gathered terms
            if (!loader)
                for (int j = tid; j < R; j += kCompute) {
                    const float4 st = reinterpret_cast<const float4 *>(sg)[j];
                    const float r = sigmoid_(fmaf(x, S[a.gs.q1a + j], st.x));
                    const float z = sigmoid_(fmaf(x, S[a.gs.q1a + R + j], st.y));
                    const float n = tanh_(fmaf(x, S[a.gs.q1a + 2 * R + j], st.z) + st.w * r);
                    va[j] = (va[j] - n) * z + n;
                }
            bar();
            SSTAMP(1);
            if (loader) loader_top(t);

            // ---- B: GRU2 (:213-214), wave u → unit u (gate rows on DPP rows 0..2)
            if (!loader) {
                const int u = wave, j = g * kSplitUnits + u;
                const float v = crit_dot<R>(S + a.gs.wih2 + (u * 3 + (row < 3 ? row : 0)) * R, va, li);
                const float *tr = RING(t);
                float gi[3], gh[3];
                if (!kPre) {
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        pq2[q] = S[a.gs.q2 + u * 3 + q];
                        pp2[q] = tr[ST_P2 + u * 3 + q];
                        pbi[q] = S[a.gs.bih2 + u * 3 + q];
                        pgh[q] = gh2[(t & 1) * 12 + u * 3 + q] + S[a.gs.bhh2 + u * 3 + q];
                    }
                    pwi0 = S[a.gs.wi0 + u];
                    pci = tr[ST_CI + u];
                    ph2 = h2own[u];
                }
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    gi[q] = (lane_bcast(v, 16 * q) + fmaf(x, pq2[q], pp2[q])) + pbi[q];
                    gh[q] = pgh[q];
                }
                const float hn = gru_gate_math(gi[0], gi[1], gi[2], gh[0], gh[1], gh[2], ph2);
                // y = (x_I + h1) + h2 (:212, :216), x_I = cI + W_I[:, 0]·x
                const float y = (fmaf(pwi0, x, pci) + va[j]) + hn;
                // y: one 128-B line per GRU workgroup (kYLine granules), so no two workgroups'
                // sc1 stores share a line (4 producers per line cost the hop ~0.5 us)
                if (lane < a.reps) publish(XG(SH_Y) + (size_t)lane * a.rep_stride + g * kYLine + u, tag, y);
                else if (lane < 2 * a.reps)
                    publish(XG(SH_H2A + (t & 1)) + (size_t)(lane - a.reps) * a.rep_stride + j, tag, hn);
                if (lane == 0) h2own[u] = hn;
                if (dbg_on && tid == 0) stamp[(t & 1) * kStamps + 2] = (unsigned)__builtin_amdgcn_s_memrealtime();
            }

            // ---- C: while fc1/fc2 run elsewhere: f2 (wave 0), step t+1's GRU1 terms (wave 1
            // publishes, wave 3 gathers), h2 → GH2 (wave 2).  The polling waves first let their y/h2
            // stores leave the CU (vmcnt(0)): polls queued behind them slow the critical y hop
            if (kDrainPub && wave != 1 && !loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (wave == 0) {
                // ---- D + E: fc3 logits (hop F2: partial sums) → MoL sample (:223-229) → x_t
                const float ul = NZ(t)[lane < 10 ? lane : 0], u10 = NZ(t)[10];
                const float s = gather_logits(tag, t);
                SSTAMP(4);
                const float xs = mol_sample_reg(s, ul, u10, lane);
                if (lane == 0) xprev[t & 1] = xs;
                SSTAMP(5);
            } else if (wave == 1) {
                if (more) {
                    const float3 v = row_dot3(S + a.gs.whh1 + (row * 3 + 0) * R, S + a.gs.whh1 + (row * 3 + 1) * R,
                                              S + a.gs.whh1 + (row * 3 + 2) * R, va, R / 4, li);
                    if (li == 0) {
                        gh1[row * 3 + 0] = v.x;
                        gh1[row * 3 + 1] = v.y;
                        gh1[row * 3 + 2] = v.z;
                    }
                    publish_terms(t + 1, false);
                }
            } else if (wave == 2) {
                if (more) {
                    auto store_h2 = [&](int, int k, float v) { vb[k] = v; };
                    gather<NG_R, kPollThreads, decltype(store_h2), kOffSleep>(
                        XG(SH_H2A + (t & 1)) + poll_off, 0, R, R, tag, a.ctl, a.timeout_ticks, t, SH_H2A + (t & 1),
                        abort_flag, lane, store_h2);
                    const float3 v = row_dot3(S + a.gs.whh2 + (row * 3 + 0) * R, S + a.gs.whh2 + (row * 3 + 1) * R,
                                              S + a.gs.whh2 + (row * 3 + 2) * R, vb, R / 4, li);
                    float *o = gh2 + ((t + 1) & 1) * 12 + row * 3;
                    if (li == 0) {
                        o[0] = v.x;
                        o[1] = v.y;
                        o[2] = v.z;
                    }
                }
            } else if (wave == 3) {
                if (more) gather_terms(t + 1);
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // loader: this step's DMA landed
            }
            bar();
            SSTAMP(3);
            if (*abort_flag) return;
        } else {
            // ---- A': y (hop Y); the gathering wave first lets its f2 stores leave the CU
            const int e = wave * 4 + row;                 // engine = fc row within the workgroup
            float pv1 = 0.0f, pv2 = 0.0f;                 // fc1 / fc2 conditioning terms (+ biases)
            if (kPre && !loader) {
                pv1 = RING(t)[ST_V1 + e];
                pv2 = RING(t)[ST_V2 + e];
            }
            if (kDrainPub && wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (wave == 0)
                gather_mapped<NG_R, kPollThreads>(XG(SH_Y) + poll_off, R, tag, a.ctl, a.timeout_ticks, t, SH_Y,
                                                  abort_flag, lane,
                                                  [](int i) { return (i / kSplitUnits) * kYLine + i % kSplitUnits; },
                                                  [&](int k, float v) { va[k] = v; });
            bar();
            SSTAMP(1);
            if (*abort_flag) return;
            if (loader) loader_top(t);
            // ---- B': fc1 (:216-218), relu → hop F1
            if (!loader) {
                const float v = crit_dot<R>(S + a.fs.w1 + e * R, va, li) + (kPre ? pv1 : RING(t)[ST_V1 + e]);
                // the 16 lanes of the engine publish replicas li, li + 16 (reps <= 32)
                for (int r = li; r < a.reps; r += 16)
                    publish(XG(SH_F1) + (size_t)r * a.rep_stride + g * kSplitFcRows + e, tag, v > 0.0f ? v : 0.0f);
                if (dbg_on && tid == 0) stamp[(t & 1) * kStamps + 6] = (unsigned)__builtin_amdgcn_s_memrealtime();
            }
            if (kDrainPub && wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // f1 stores out first
            if (wave == 0)
                gather<NG_F, kPollThreads>(XG(SH_F1) + poll_off, 0, F, F, tag, a.ctl, a.timeout_ticks, t, SH_F1,
                                           abort_flag, lane, [&](int, int k, float v) { vb[k] = v; });
            bar();
            SSTAMP(2);
            if (*abort_flag) return;
            // ---- C': fc2 (:220-221), relu → the own 16 rows of f2 (LDS)
            if (!loader) {
                const float v = crit_dot<F>(S + a.fs.w2 + e * F, vb, li) + (kPre ? pv2 : RING(t)[ST_V2 + e]);
                if (li == 0) f2[e] = v > 0.0f ? v : 0.0f;
            }
            if (loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
            SSTAMP(3);
            if (*abort_flag) return;
            // ---- D': fc3 partial logits over the own f2 rows (:223) → hop F2; compute wave k
            // publishes replicas k, k + 4, …  The FC workgroups need no x: on to the next y.
            if (!loader && lane < NC) {
                const float *w3p = S + a.fs.w3p + lane;
                float p = 0.0f;
#pragma unroll
                for (int k = 0; k < kSplitFcRows; ++k) p = fmaf(w3p[k * kSplitLogitLine], f2[k], p);
                for (int r = wave; r < a.reps; r += kWaves)
                    publish(XG(SH_F2) + (size_t)r * a.rep_stride + g * kSplitLogitLine + lane, tag, p);
            }
            if (dbg_on && tid == 0) stamp[(t & 1) * kStamps + 7] = (unsigned)__builtin_amdgcn_s_memrealtime();
            continue;
        }
        x = xprev[t & 1];   // sampled by wave 0 in phase C
    }
    __syncthreads();
    if (w == 0 && tid == 0) a.out[(size_t)a.b0 * a.L + (t_end - 1)] = xprev[(t_end - 1) & 1];
    // carry the recurrent state to the next time chunk
    float *st = a.state + (size_t)w * split_state_w(R);
    for (int i = tid; i < R; i += kThreads) {
        st[i] = va[i];
        st[R + i] = vb[i];
    }
    if (gru)
        for (int i = tid; i < RT; i += kThreads) st[2 * R + i] = sg[i];
    if (tid < 24) st[6 * R + tid] = gh2[tid];
    if (tid < 4) st[6 * R + 24 + tid] = h2own[tid];
    if (tid == 0) st[6 * R + 28] = xprev[(t_end - 1) & 1];
}

#define WRNN_K_SPLIT512 fatchord_split_kernel<512, 512, false>
#define WRNN_K_SPLIT512_DBG fatchord_split_kernel<512, 512, true>

bool split_has_kernel(int R, int F) { return R == 512 && F == 512; }

hipError_t launch_split(const SplitArgs &a, size_t lds_bytes, hipStream_t st) {
    SplitArgs args = a;
    void *params[] = {&args};
    const void *k = a.dbg ? (const void *)WRNN_K_SPLIT512_DBG : (const void *)WRNN_K_SPLIT512;
    return hipLaunchKernel(k, dim3(a.Gg + a.Gf), dim3(kThreads), params, lds_bytes, st);
}

hipError_t prepare_split_kernel(int max_lds_bytes) {
    for (const void *k : {(const void *)WRNN_K_SPLIT512, (const void *)WRNN_K_SPLIT512_DBG}) {
        hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds_bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t split_occupancy(int *blocks_per_cu, size_t lds_bytes) {
    int best = 1 << 30;
    for (const void *k : {(const void *)WRNN_K_SPLIT512, (const void *)WRNN_K_SPLIT512_DBG}) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kThreads, lds_bytes);
        if (e != hipSuccess) return e;
        best = n < best ? n : best;
    }
    *blocks_per_cu = best;
    return hipSuccess;
}

}  // namespace wrnn
