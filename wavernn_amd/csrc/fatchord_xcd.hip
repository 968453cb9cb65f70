// fatchord_xcd.hip — XCD-resident persistent kernel for MoL rows (rnn 512, fc 512): the sample
// loop of models/fatchord_version.py:201-241 for ONE row on the 32 CUs of ONE XCD, up to eight
// rows (one per XCD) per launch.
//
// Why one XCD: every hand-off of the loop is an all-gather among the workgroups that hold the
// weights.  Kept inside one XCD, a granule can be published with a PLAIN store — the line stays
// in that XCD's L2, where the consumers' sc1 polls find it — instead of an sc1 store that goes
// to the Infinity Fabric: tools/xcdbench.hip measures 0.23 µs one-way (0.41 sc1 same-XCD, 0.59
// cross-XCD), tools/xcdhop.hip 0.50 µs per 32 → 32 all-gather hop (1.16 spread over 8 XCDs).
// The 11.4 MB of loop weights fit the XCD's 32 CUs as 96 KB of W_hh1 per CU in LDS and the rest
// (W_ih2, fc1, fc2 rows, fc3 columns, W_hh2) in the VGPRs of 8 waves (two per SIMD).
//
// Workgroup c of an XCD owns GRU units 16c..16c+15 (both GRUs) and fc rows 16c..16c+15; wave w
// of it units / fc rows 16c + 2w + {0, 1}.  Per step t (x = x_{t-1}):
//   B1 → GRU1 for ALL units, one per thread, from the gathered terms S (rank-1 in x: no hop)
//   B2 → W_ih2·h1 for the wave's 6 gate rows (VGPR weights, h1 from LDS) → GRU2 gates → publish
//        y = x_I + h1 + h2 and h2                                                  [hop Y]
//   B3 → fc1 rows (2 per wave) → relu → publish f1                               [hop F1]
//   B4 → fc2 rows → relu → fc3 partial logits of the workgroup's 16 f2 rows → B5 → wave 0 sums
//        the 8 waves' partials → publish 30 partials                             [hop F2]
//   wave 0 gathers all 32 × 30 partials, sums + b3, samples (MoL, utils/distribution.py:87-123,
//   redundantly and bit-identically in every workgroup) → x_t.
// Off the critical path, waves 1..7: W_hh1·h1 (LDS weights) → the GRU1 terms of step t+1 →
// publish (hop S, double-buffered), gather h2 (wave 6) → W_hh2·h2 (VGPR weights) for the next
// GRU2, gather S (waves 1, 2, 5 and fc2 wave 4, a quarter each), the conditioning terms and
// noise of step t+2 into the LDS ring (wave 7).
//
// Membership: each workgroup reads its XCC id from the hardware register and takes an index
// from a per-XCD arrival counter, so correctness never depends on the dispatcher's placement
// (a missing member shows up as a bounded-wait timeout, never as a hang).  Arithmetic is fp32
// with the sums re-associated (tolerance-checked against the oracle like the other kernels).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fatchord_loop.h"
#include "fatchord_xcd.h"
#include "wrnn_device.h"
#include "xcd_device.h"

namespace wrnn {

// diagnostics (tools/ab_libs.sh): skip an off-critical exchange (wrong results, timing only)
#ifndef WRNN_XCD_SKIP_SG
#define WRNN_XCD_SKIP_SG 0
#endif
#ifndef WRNN_XCD_SKIP_H2
#define WRNN_XCD_SKIP_H2 0
#endif
// diagnostics: 1 = skip ALL the off-critical recurrent work (W_hh1·h1 → the GRU1 terms S and
// their exchange, the h2 exchange, W_hh2·h2): the critical path alone, timing only — the ceiling
// of moving that work off this XCD (DESIGN.md §9.1's two-XCD-per-row idea)
#ifndef WRNN_XCD_SKIP_RECUR
#define WRNN_XCD_SKIP_RECUR 0
#endif
#ifndef WRNN_XCD_PRIO
#ifndef WRNN_XCD_RS
#define WRNN_XCD_RS 1           // GRU2's three engine dots reduce-scattered (e32dot3_rs; 0: three e32dot, A/B)
#endif
#define WRNN_XCD_PRIO 0         // s_setprio of wave 0 (the poller / sampler)
#endif

// the wave that gathers the fourth quarter of the next step's GRU1 terms: 4 (an fc2 wave, idle
// after its fc3 hand-off) — wave 6 gathered it after h2, and its W_hh2·h2 then ended with the
// sampler (both at the step-end barrier); 6: as before, 3: the other fc2 wave (A/B)
#ifndef WRNN_XCD_SQ3_WAVE
#define WRNN_XCD_SQ3_WAVE 4
#endif
// y and h2 published per wave: lane 0 stores both engines' units (lanes 0 and 32 before, one in
// each half of the wave) as one 16-byte pair — 1 row 3.36-3.37 → 3.31-3.33 µs/step,
// profiles/r05_ab_xcd_pub16.log (the same pairing of the f1 rows / fc3 partials, already adjacent
// lanes of one store: slower, not kept); 0: per engine (A/B)
#ifndef WRNN_XCD_PUB16
#define WRNN_XCD_PUB16 1
#endif
#ifndef WRNN_XCD_STAMP_W13
#define WRNN_XCD_STAMP_W13 5    // stamped builds: the wave whose W_hh2·h2 end is stamp 13 (6: the h2 gatherer)
#endif
#define XSTAMPW(kk, w)                                                                                        \
    do {                                                                                                      \
        if (kDbg && a.dbg && wave == (w) && lane == 0 && t - a.t0 < a.dbg_steps &&                            \
            (!WRNN_XCD_BAR_STAMPS || ((kk) != 3 && ((kk) < 9 || (kk) > 14))))                                 \
            a.dbg[((size_t)mem * a.dbg_steps + (t - a.t0)) * kStamps + (kk)] = (unsigned)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define XSTAMP(kk) XSTAMPW(kk, 0)
// diagnostics (WRNN_XCD_BAR_STAMPS): waves 1..6 → stamps 9..14, wave 7 → stamp 3, at the step-end barrier
#define XSTAMP_BAR()                                                                                          \
    do {                                                                                                      \
        if (WRNN_XCD_BAR_STAMPS && kDbg && a.dbg && wave > 0 && lane == 0 && t - a.t0 < a.dbg_steps)          \
            a.dbg[((size_t)mem * a.dbg_steps + (t - a.t0)) * kStamps + (wave == 7 ? 3 : 8 + wave)] =          \
                (unsigned)__builtin_amdgcn_s_memrealtime();                                                   \
    } while (0)

template <bool kDbg>
__global__ __launch_bounds__(kXThreads, 2) void fatchord_xcd_kernel(XcdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int R = 512, TW = kXcdWgs * kXTerms;
    const XcdLds ll = xcd_lds_layout();
    const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, eng = lane >> 5;
    // the wave index wave-uniform (SGPR): its role branches become scalar, its offsets scalar operands
    const int wave = WRNN_XCD_UNIFORM_WAVE ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
    float *whh1 = smem + ll.whh1, *whh2l = smem + ll.whh2, *f2x = smem + ll.f2x, *h1s = smem + ll.h1, *h2s = smem + ll.h2, *sg = smem + ll.sg, *w3s = smem + ll.w3;
    float *ring = smem + ll.ring, *nzr = smem + ll.nz, *gh2s = smem + ll.gh2, *cst = smem + ll.cst, *xs = smem + ll.xs;
    int *misc = reinterpret_cast<int *>(smem + ll.misc);
    int *abort_flag = misc, *h2ready = misc + 2, *f2ready = misc + 3, *ygot = misc + 4, *f1got = misc + 5;

    // ---- membership: XCD k (row b0 + k) and index c within it
    if (tid == 0) {
        const int k = (int)xcc_id();
        int c = kXcdWgs;
        if (k < a.nb) c = atomicAdd(&a.members[k], 1);
        misc[1] = (k < a.nb && c < kXcdWgs) ? k * kXcdWgs + c : -1;
        misc[0] = 0;
        for (int i = 2; i < 8; ++i) misc[i] = 0;
    }
    if (tid < 64) f2x[tid] = 0.0f;   // the fc3 hand-off pairs: tag 0, which no step carries
    __syncthreads();
    const int mem = __builtin_amdgcn_readfirstlane(misc[1]);   // wave-uniform: hop addresses in SGPRs
    if (mem < 0) return;
    const int k = mem / kXcdWgs, c = mem - k * kXcdWgs;
    const int b = a.b0 + k;
    const int t_end = a.t0 + a.Lc;
    const int t_terms = min(t_end, a.L - 1);
    unsigned long long *xg = a.xg + (size_t)k * kXXcdStride;
    auto XG = [&](int hop) { return xg + (size_t)hop * kXHopStride; };
    // publishes through one wave-uniform buffer descriptor + a 32-bit granule index (the 64-bit
    // per-lane pointers of each hop stayed live across the loop and were spilled: the F2 publish
    // reloaded its address from scratch and waited vmcnt(0) on the critical path)
    const __amdgpu_buffer_rsrc_t xgr = __builtin_amdgcn_make_buffer_rsrc(xg, 0, 0x7fffffff, 0x00020000);
    auto XGI = [&](int hop) { return hop * (int)kXHopStride; };
    auto RING = [&](int t) { return ring + (t & (kXRing - 1)) * kXTerms; };
    auto NZ = [&](int t) { return nzr + (t & (kXRing - 1)) * kXNoise; };
    auto TERMS = [&](int t) { return a.terms + ((size_t)(t - a.t0) * a.nb + k) * TW + (size_t)c * kXTerms; };
    const float *S = a.slab + (size_t)c * a.s.total;
    const unsigned long long prow = (unsigned long long)(a.row0 + k);

    // ---- register-resident weights
    //   wih2 (all waves): GRU2 pass q = gate q of unit ui = 2w + e, chunks li + 32m of the row
    //   wr (one register set, contents by role):
    //     waves 1, 2 / 3, 4: fc1 / fc2 rows 8h + r, r = 0..7, at the granules this lane polls (fc8_rows)
    //     waves 5..7: W_hh2 rows 8(w − 5) + 2p + e, p = 0..3, at wr[4p + m] (32-lane chunks)
    //     wave 0: wr[0..7] the F2 poll buffer, wr[8..15] W_hh2 rows 24 + 2p + e, p = 0..1
    f4v wih2[3][4], wr[16];
    auto ldrow = [&](const float *row, int m) { return *reinterpret_cast<const f4v *>(row + 4 * (li + 32 * m)); };
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int q = 0; q < 3; ++q) wih2[q][m] = ldrow(S + a.s.wih2 + (wave * 6 + 2 * q + eng) * R, m);
    const bool fcw = wave >= kXWaveFc1 && wave < kXWaveFc2 + 2;
    if (fcw) {
        const int hf = (wave - kXWaveFc1) & 1;
        const float *W = S + (wave < kXWaveFc2 ? a.s.w1 : a.s.w2) + hf * 8 * R;
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const f2v lo = *reinterpret_cast<const f2v *>(W + r * R + 2 * (lane + 64 * (2 * hh)));
                const f2v hi = *reinterpret_cast<const f2v *>(W + r * R + 2 * (lane + 64 * (2 * hh + 1)));
                wr[2 * r + hh] = f4v{lo.x, lo.y, hi.x, hi.y};
            }
    } else {
        const int rb = wave == 0 ? 24 - 4 : 8 * (wave - 5);   // wave 0: passes 2, 3 → rows 24..27
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int m = 0; m < 4; ++m)
                wr[4 * p + m] = (wave != 0 || p >= 2) ? ldrow(S + a.s.whh2 + (rb + 2 * p + eng) * R, m)
                                                      : f4v{0.0f, 0.0f, 0.0f, 0.0f};
    }
    // GRU1 of unit tid: x-coefficients
    const float q1r = S[a.s.q1a + tid], q1z = S[a.s.q1a + R + tid], q1n = S[a.s.q1a + 2 * R + tid];
    const int ui = wave * 2 + eng;                   // this engine's local GRU unit
    // W_hh1 rows (waves 0, 3, 4, 5: ten each, wave 7: eight): gh0 + 2p + e, p = 0..4; lane li < 5
    // of an engine publishes the terms of its row gh0 + 2·li + e
    const bool gh1w = wave == 0 || wave == 3 || wave == 4 || wave == 5 || wave == 7;
    const int gh0 = wave == 0 ? 0 : wave == 7 ? 40 : 10 * (wave - 2);
    // sampler noise of step t → NZ(t): u1 → log(-log u1) (distribution.py:107), u2 → log u2 − log(1 − u2) (:119)
    auto noise_term = [&](int t) -> float {
        float uu;
        if (a.noise) uu = a.noise[((size_t)t * a.Bt + b) * 11 + lane];
        else uu = philox_noise(a.seed, prow, (uint32_t)t, (uint32_t)lane, 1);
        return mol_noise_term(uu, lane);
    };
    // GRU1 term(s) of step t for W_hh1 row rr (u·3 + q), by lane 0 / 32 of an engine:
    //   q = 0: S_r = (GH1_r + b_hh,r) + (P1_r + b_ih,r), q = 1: S_z likewise,
    //   q = 2: Gh_n = GH1_n + b_hh,n (term 3) and Gi_n = P1_n + b_ih,n (term 2)
    auto publish_term = [&](int t, int rr, float gh) {
        const int u = rr / 3, q = rr - 3 * u;
        const float p1 = RING(t)[XT_P1 + rr], bh = cst[XC_BHH1 + rr], bi = cst[XC_BIH1 + rr];
        const int g = XGI(XH_S0 + (t & 1)) + (c * kXUnits + u) * 4;
        const uint32_t tag = (uint32_t)t + 1u;
        if (q < 2) {
            xpub_b(xgr, g + q, tag, (gh + bh) + (p1 + bi));
        } else {
            xpub_b(xgr, g + 3, tag, gh + bh);
            xpub_b(xgr, g + 2, tag, p1 + bi);
        }
    };
    // the GRU1 terms of this wave's W_hh1 rows (gh[p]: row gh0 + 2p + e), lanes li < 5
    auto publish_terms = [&](int t, const float (&gh)[5]) {
        const int rr = gh0 + 2 * li + eng;
        if (li < 5 && rr < 48) {
            const float v = li == 0 ? gh[0] : li == 1 ? gh[1] : li == 2 ? gh[2] : li == 3 ? gh[3] : gh[4];
            publish_term(t, rr, v);
        }
    };
    // W_hh1·h1 for this wave's rows (the GRU1 terms of step t + 1, published later by
    // publish_terms): all dots first, so LDS reads of later rows overlap earlier dots
    auto gh1_dots = [&](float (&gh)[5]) {
        f4v hx[4];
        e32x(h1s, li, hx);
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            f4v w4[4];
            e32x(whh1 + min(gh0 + 2 * p + eng, 47) * R, li, w4);
            gh[p] = e32dot(w4, hx);
        }
    };
    // intra-workgroup step flags in LDS (no data behind them, or the writer drained its LDS
    // stores first): the critical waves mark "y gathered" / "f1 gathered", the others wait for
    // them so that their own memory traffic stays out of the critical hops' windows
    auto set_flag = [&](int *f, uint32_t tag) {
        if (lane == 0) __hip_atomic_store(f, (int)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto wait_flag = [&](int *f, uint32_t tag) {
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)tag)
            __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
    };
    // W_hh2·h2 → gh2s for the next GRU2 (after wave 6 has gathered h2): lanes li < np store the
    // rows rb + 2·li + e
    auto gh2_store = [&](int rb, int np, const float (&gh)[5]) {
        const int rr = rb + 2 * li + eng;
        if (li < np) gh2s[rr] = li == 0 ? gh[0] : li == 1 ? gh[1] : li == 2 ? gh[2] : li == 3 ? gh[3] : gh[4];
    };
    // a quarter of step t's GRU1 terms (waves 1, 2, 5, WRNN_XCD_SQ3_WAVE: 512 granules each, one
    // poll round)
    auto gather_terms = [&](int t) {
        const int qq = wave == 1 ? 0 : wave == 2 ? 1 : wave == 5 ? 2 : 3;
        xgather16<4>(XG(XH_S0 + (t & 1)) + qq * 512, (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t, XH_S0 + (t & 1),
                     abort_flag, lane, [&](int i, float v0, float v1) {
                         *reinterpret_cast<f2v *>(sg + qq * 512 + i) = f2v{v0, v1};
                     });
    };

    // ---- prologue: W_hh1, fc3 columns, small vectors, ring slots t0..t0+2, state
    {
        const f4v *src = reinterpret_cast<const f4v *>(S + a.s.whh1);
        f4v *dst = reinterpret_cast<f4v *>(whh1);
        for (int i = tid; i < 48 * R / 4; i += kXThreads) dst[i] = src[i];
        src = reinterpret_cast<const f4v *>(S + a.s.whh2 + kXH2RegRows * R);
        dst = reinterpret_cast<f4v *>(whh2l);
        for (int i = tid; i < (48 - kXH2RegRows) * R / 4; i += kXThreads) dst[i] = src[i];
        for (int i = tid; i < kXFcRows * 32; i += kXThreads) w3s[i] = S[a.s.w3 + i];
        for (int i = tid; i < kXCst; i += kXThreads) cst[i] = S[a.s.cst + i];
        for (int t = a.t0; t < a.t0 + 3; ++t) {
            if (t <= t_terms)
                for (int i = tid; i < kXTerms; i += kXThreads) RING(t)[i] = TERMS(t)[i];
            if (wave == 1 && lane < 11 && t < a.L) NZ(t)[lane] = noise_term(t);
        }
    }
    const bool resume = a.t0 > 0;
    float *st = a.state + ((size_t)k * kXcdWgs + c) * kXStateW;
    float h1v = resume ? st[tid] : 0.0f;              // h1 of unit tid (recurrent, this thread)
    float h2own = resume ? st[512 + 2048 + 48 + ui] : 0.0f;   // h2 of this engine's unit
    // consume the carried-state loads here (an empty asm use: the wait lands before the loop);
    // left pending into the loop, their first use inside it is an s_waitcnt vmcnt(0) in EVERY
    // step (GRU1's h1 update), draining all the wave's in-flight publishes and loads there
    asm volatile("" : "+v"(h1v), "+v"(h2own));
    if (resume) {
        for (int i = tid; i < 4 * R; i += kXThreads) sg[i] = st[512 + i];
        if (tid < 48) gh2s[tid] = st[512 + 2048 + tid];
        if (tid == 0) xs[(a.t0 + 1) & 1] = st[512 + 2048 + 48 + 16];
    } else {
        if (tid < 48) gh2s[tid] = 0.0f;
        if (tid == 0) xs[1] = 0.0f;
    }
    __syncthreads();
    if (!resume) {   // GRU1 terms of step 0 (GH1 = 0), published and gathered
        if (gh1w) {
            const float z5[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
            publish_terms(0, z5);
        }
        if (wave == 1 || wave == 2 || wave == 5 || wave == WRNN_XCD_SQ3_WAVE) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            gather_terms(0);
        }
    }
    __syncthreads();
    if (*abort_flag) return;

    if (WRNN_XCD_PRIO && wave == 0) __builtin_amdgcn_s_setprio(WRNN_XCD_PRIO);
    float x = xs[(a.t0 + 1) & 1];                    // x_{t-1}, wave-uniform
    f4v s4 = lds4(sg + 4 * tid);                     // GRU1 terms of unit tid for step t
    for (int t = a.t0; t < t_end; ++t) {
        const uint32_t tag = (uint32_t)t + 1u;
        const bool more = t + 1 < a.L;
        const float *tr = RING(t);
        XSTAMP(0);
        if (kDbg && a.dbg && wave == 0 && lane == 0 && t - a.t0 < a.dbg_steps)   // shader clock beside the 100 MHz one
            a.dbg[((size_t)mem * a.dbg_steps + (t - a.t0)) * kStamps + 15] = (unsigned)__builtin_amdgcn_s_memtime();
        // operands of the GRU2 gate math (engine unit ui): LDS reads issued before GRU1's
        // transcendental chain (behind its h1 store the compiler could not move them)
        float q2v[3], p2v[3], bi2[3], ghv[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            q2v[q] = cst[XC_Q2 + ui * 3 + q];
            p2v[q] = tr[XT_P2 + ui * 3 + q];
            bi2[q] = cst[XC_BIH2 + ui * 3 + q];
            ghv[q] = gh2s[ui * 3 + q] + cst[XC_BHH2 + ui * 3 + q];
        }
        const float wi0v = cst[XC_WI0 + ui], civ = tr[XT_CI + ui];
        // ---- GRU1 (:208-210), unit tid
        {
            const float r = sigmoid_(fmaf(x, q1r, s4.x));
            const float z = sigmoid_(fmaf(x, q1z, s4.y));
            const float n = tanh_(fmaf(x, q1n, s4.z) + s4.w * r);
            h1v = (h1v - n) * z + n;
            h1s[tid] = h1v;
        }
        float p2q[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) p2q[q] = fmaf(x, q2v[q], p2v[q]) + bi2[q];
        const float xi = fmaf(wi0v, x, civ);   // x_I of unit ui
        bar();
        XSTAMP(1);
        // ---- GRU2 (:212-214): pass q → gate q of unit ui (W_ih2[:, :R]·h1), all lanes of the engine
        {
            f4v hx[4];
            e32x(h1s, li, hx);
            // x_I + h1 of the engine's unit (:212) formed before the dots and pinned there: hipcc
            // otherwise sinks the h1 LDS read into the publishing lane's branch after the gate math
            float yb = xi + h1s[c * kXUnits + ui];
            asm volatile("" : "+v"(yb));
            float g_r, g_z, g_n;   // valid in lanes li == 0 (the publishing lane)
            if (WRNN_XCD_RS) {
                e32dot3_rs(wih2[0], wih2[1], wih2[2], hx, lane, g_r, g_z, g_n);
            } else {
                g_r = e32dot(wih2[0], hx);
                g_z = e32dot(wih2[1], hx);
                g_n = e32dot(wih2[2], hx);
            }
            const float hn = gru_gate_math(g_r + p2q[0], g_z + p2q[1], g_n + p2q[2], ghv[0], ghv[1], ghv[2], h2own);
            h2own = hn;
            // y = (x_I + h1) + h2 (:212, :216)
            const float y = yb + hn;
            if (WRNN_XCD_PUB16) {   // both engines' granules (units 2w, 2w + 1) in one 16-byte store
                const float y1 = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(y), 32));
                if (lane == 0)
                    __builtin_amdgcn_raw_buffer_store_b128(u4v{__float_as_uint(y), tag, __float_as_uint(y1), tag}, xgr,
                                                           (XGI(XH_Y) + c * kXUnits + 2 * wave) * 8, 0, 0);
            } else if (li == 0) {
                xpub_b(xgr, XGI(XH_Y) + c * kXUnits + ui, tag, y);   // h2: after hop Y (pub_h2)
            }
        }
        XSTAMP(2);
        // Off-critical memory traffic (GRU1-term and h2 publishes, the S / h2 gathers, the ring)
        // waits for the critical waves' flags: hop Y's window (GRU2 → y gathered) carries only y,
        // hop F1's only f1, hop F2's only the partials (a second poll stream or a burst of stores
        // beside a critical poll costs it ≈ 0.2 µs: tools/xcdhop.hip PACED variants).
        //   after y gathered  : publish the GRU1 terms of step t+1 and h2
        //   after f1 gathered : gather h2 (wave 6), S (waves 1, 2, 5, 6), the ring (wave 7)
        //   after h2 gathered : W_hh2·h2 (waves 0, 1, 2, 5, 6, 7)
        auto pub_h2 = [&]() {
            if (WRNN_XCD_PUB16) {
                const float h1o = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(h2own), 32));
                if (lane == 0)
                    __builtin_amdgcn_raw_buffer_store_b128(u4v{__float_as_uint(h2own), tag, __float_as_uint(h1o), tag},
                                                           xgr, (XGI(XH_H2) + c * kXUnits + 2 * wave) * 8, 0, 0);
            } else if (li == 0) {
                xpub_b(xgr, XGI(XH_H2) + c * kXUnits + ui, tag, h2own);
            }
        };
        // fc waves: lane l ends fc8_rows with row 8h + j + 2·(l >> 4) in o[j]; lanes with
        // (l & 15) < 2 publish row 8h + (l & 1) + 2·(l >> 4)
        const int jq = lane & 1, rho = jq + 2 * (lane >> 4);
        if (wave == 0) {
            if (more && !WRNN_XCD_SKIP_RECUR) {
                float gh[5];
                gh1_dots(gh);
                wait_flag(ygot, tag);
                publish_terms(t + 1, gh);
                pub_h2();
                wait_flag(h2ready, tag);
                f4v hx[4];
                e32x(h2s, li, hx);
                float g2[5] = {e32dot(*reinterpret_cast<const f4v(*)[4]>(&wr[8]), hx),
                               e32dot(*reinterpret_cast<const f4v(*)[4]>(&wr[12]), hx), 0.0f, 0.0f, 0.0f};
                gh2_store(24, 2, g2);
            }
            // ---- hop F2: Σ of the 32 workgroups' partials + b3 → sample
            // lane l: logits (2jp, 2jp+1), jp = l & 15, of producers 8·(l >> 4) + m, m = 0..7:
            // one 16-byte load each (256 B apart: immediates)
            const int jp = lane & 15, pg = lane >> 4;
            const float ua = NZ(t)[jp < 5 ? 2 * jp : 0], ub = NZ(t)[jp < 5 ? 2 * jp + 1 : 0], u10 = NZ(t)[10];
            const float b3a = cst[XC_B3 + 2 * jp], b3b = cst[XC_B3 + 2 * jp + 1];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const __amdgpu_buffer_rsrc_t rf = hop_rsrc(XG(XH_F2));
            const int goff = pg * 8 * kXF2Line * 8 + jp * 16;
            const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
            unsigned spins = 0;
            // the polled pieces live in wr[0..7] (wave 0 holds no weights there), polled in place
            // and read after the loop (the abort path zeroes them there: no copies on the exit)
            u4v *v = reinterpret_cast<u4v *>(&wr[0]);
            for (;;) {
#pragma unroll
                for (int m = 0; m < 8; ++m) v[m] = ld16_sc1(rf, goff + m * kXF2Line * 8);
                bool ok = true;
#pragma unroll
                for (int m = 0; m < 8; ++m) ok &= (v[m].y == tag) & (v[m].w == tag);
                if (__ballot(!ok) == 0) break;   // wave-uniform exit: no exec-mask branches
                if ((++spins & 63u) == 0) {
                    const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                    const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    if (late || other) {
                        if (late) record_abort(a.ctl, -4, t, XH_F2, blockIdx.x);
                        *abort_flag = 1;
#pragma unroll
                        for (int m = 0; m < 8; ++m) v[m] = u4v{0u, 0u, 0u, 0u};
                        break;
                    }
                }
            }
            float pa[8], pb[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                pa[m] = __uint_as_float(v[m].x);
                pb[m] = __uint_as_float(v[m].z);
            }
            XSTAMP(7);
#pragma unroll
            for (int n = 4; n >= 1; n /= 2)
#pragma unroll
                for (int m = 0; m < n; ++m) {
                    pa[m] += pa[m + n];
                    pb[m] += pb[m + n];
                }
            // + the other producer groups (lanes l ^ 16, l ^ 32): identical bits in all four
            cross_rows_pair(pa[0], pb[0]);
            const float la = pa[0] + b3a, lb = pb[0] + b3b;   // logits 2jp, 2jp+1
            x = mol_sample_pairs(la, lb, ua, ub, u10, jp);
            if (lane == 0) {
                xs[t & 1] = x;
                if (c == 0) a.out[(size_t)b * a.L + t] = x;
            }
            XSTAMP(8);
        } else if (wave < kXWaveFc2) {
            // ---- hop Y → fc1 (:216-218) rows 8h.. in registers → relu → hop F1
            const int hf = wave - kXWaveFc1, rg = 8 * hf + rho;
            const float v1 = tr[XT_V1 + rg];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u4v v[4];
            xpoll16<4>(XG(XH_Y), tag, a.ctl, a.timeout_ticks, t, XH_Y, abort_flag, lane, v);
            if (hf == 0) set_flag(ygot, tag);
            XSTAMPW(3, 1);
            f2v yk[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) yk[kk] = f2v{__uint_as_float(v[kk].x), __uint_as_float(v[kk].z)};
            float o[2];
            fc8_rows(wr, yk, o);
            const float A = (jq == 0 ? o[0] : o[1]) + v1;
            if ((lane & 15) < 2) xpub_b(xgr, XGI(XH_F1) + c * kXFcRows + rg, tag, A > 0.0f ? A : 0.0f);
            XSTAMPW(4, 1);
            if (more && !WRNN_XCD_SKIP_RECUR) {   // h2 out; after f1 gathered: a quarter of the next S; W_hh2 LDS rows 28 + 10h + 2p + e
                pub_h2();
                wait_flag(f1got, tag);
                if (!WRNN_XCD_SKIP_SG) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    gather_terms(t + 1);
                }
                wait_flag(h2ready, tag);
                f4v hx[4];
                e32x(h2s, li, hx);
                float gh[5];
#pragma unroll
                for (int p = 0; p < 5; ++p) {
                    f4v w4[4];
                    e32x(whh2l + (10 * hf + 2 * p + eng) * R, li, w4);
                    gh[p] = e32dot(w4, hx);
                }
                gh2_store(kXH2RegRows + 10 * hf, 5, gh);
                XSTAMPW(11, 1);
            }
        } else if (wave < kXWaveFc2 + 2) {
            const int hf = wave - kXWaveFc2;
            if (more && !WRNN_XCD_SKIP_RECUR) {   // W_hh1 rows; after y gathered their terms and h2 out
                float gh[5];
                gh1_dots(gh);
                wait_flag(ygot, tag);
                publish_terms(t + 1, gh);
                pub_h2();
            }
            XSTAMPW(9, 3);
            // ---- hop F1 → fc2 (:220-221) rows 8h.. in registers → relu → fc3 partial logits of
            // those rows (:223); wave 4 hands its partials to wave 3 (LDS flag), wave 3 publishes
            // the workgroup's 32 (hop F2)
            float v2[2], w3c[8];
#pragma unroll
            for (int j = 0; j < 2; ++j) v2[j] = tr[XT_V2 + 8 * hf + j + 2 * (lane >> 4)];
#pragma unroll
            for (int r = 0; r < 8; ++r) w3c[r] = w3s[(8 * hf + r) * 32 + li];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u4v v[4];
            xpoll16<4>(XG(XH_F1), tag, a.ctl, a.timeout_ticks, t, XH_F1, abort_flag, lane, v);
            if (hf == 0) set_flag(f1got, tag);
            XSTAMPW(5, 3);
            f2v fk[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) fk[kk] = f2v{__uint_as_float(v[kk].x), __uint_as_float(v[kk].z)};
            float o[2];
            fc8_rows(wr, fk, o);
            float p = 0.0f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float f = o[j] + v2[j];
                const float f2 = f > 0.0f ? f : 0.0f;
#pragma unroll
                for (int g = 0; g < 4; ++g) p = fmaf(w3c[j + 2 * g], lane_bcast(f2, 16 * g), p);
            }
            // wave 4 → wave 3: 8-byte (value, tag) pairs in LDS, polled by the consumer lanes
            // themselves (one LDS round trip less than data + flag + a flag poll)
            unsigned long long *f2p = reinterpret_cast<unsigned long long *>(f2x);
            if (hf == 1) {
                if (lane < 32)
                    __hip_atomic_store(f2p + lane, ((unsigned long long)tag << 32) | __float_as_uint(p), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                // wave 4 stores on every path (its poll is bounded); the abort word ends the wait
                // too should that ever change
                unsigned spin = 0;
                unsigned long long pv = (unsigned long long)tag << 32;
                for (;;) {
                    if (lane < 32) pv = __hip_atomic_load(f2p + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (__ballot((uint32_t)(pv >> 32) != tag) == 0) break;
                    if ((++spin & 255u) == 0 &&
                        __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                        break;
                }
                if (lane < kXF2Line)   // 30, 31: zero weights
                    xpub_b(xgr, XGI(XH_F2) + c * kXF2Line + lane, tag, p + __uint_as_float((uint32_t)pv));
                XSTAMPW(6, 3);
            }
            // the fourth quarter of the next step's GRU1 terms (this wave has polled F1 itself:
            // the hop F1 window is over)
            if ((WRNN_XCD_SQ3_WAVE == 3 || WRNN_XCD_SQ3_WAVE == 4) && wave == WRNN_XCD_SQ3_WAVE && more &&
                !WRNN_XCD_SKIP_RECUR && !WRNN_XCD_SKIP_SG) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                gather_terms(t + 1);
            }
        } else if (more) {
            // ---- waves 5..7: W_hh1 rows (5, 7) → after y gathered their terms and h2 out; after
            // f1 gathered: h2 (wave 6, then flag), an S quarter (5; 6 with WRNN_XCD_SQ3_WAVE 6),
            // the ring (7); after h2 gathered: W_hh2·h2 (VGPR rows)
            if (WRNN_XCD_SKIP_RECUR) {
                if (wave == 7) {
                    wait_flag(f1got, tag);
                    if (t + 2 >= a.t0 + 3) {
                        if (t + 2 <= t_terms && lane < kXTerms / 4)
                            reinterpret_cast<f4v *>(RING(t + 2))[lane] = reinterpret_cast<const f4v *>(TERMS(t + 2))[lane];
                        if (t + 2 < a.L && lane < 11) NZ(t + 2)[lane] = noise_term(t + 2);
                    }
                }
                goto step_end;
            }
            if (wave != 6) {
                float gh[5];
                gh1_dots(gh);
                wait_flag(ygot, tag);
                publish_terms(t + 1, gh);
            } else {
                wait_flag(ygot, tag);
            }
            pub_h2();
            wait_flag(f1got, tag);
            if (wave == 6) {
                if (!WRNN_XCD_SKIP_H2) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    xgather16<4>(XG(XH_H2), tag, a.ctl, a.timeout_ticks, t, XH_H2, abort_flag, lane,
                                 [&](int i, float v0, float v1) { *reinterpret_cast<f2v *>(h2s + i) = f2v{v0, v1}; });
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                set_flag(h2ready, tag);
                XSTAMPW(10, 6);
            }
            if (wave <= 6) {
                if (!WRNN_XCD_SKIP_SG && (wave == 5 || WRNN_XCD_SQ3_WAVE == 6)) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    gather_terms(t + 1);
                }
                XSTAMPW(14, 5);
            } else if (t + 2 >= a.t0 + 3) {
                // ring: step t+2's terms and sampler noise, loaded and stored within this window
                // (a load carried across steps in registers would not fit the VGPR budget, and an
                // LDS-DMA makes hipcc wait for it before every later LDS access of the issuing wave)
                if (t + 2 <= t_terms && lane < kXTerms / 4)
                    reinterpret_cast<f4v *>(RING(t + 2))[lane] = reinterpret_cast<const f4v *>(TERMS(t + 2))[lane];
                if (t + 2 < a.L && lane < 11) NZ(t + 2)[lane] = noise_term(t + 2);
                XSTAMPW(12, 7);
            }
            wait_flag(h2ready, tag);
            {
                f4v hx[4];
                e32x(h2s, li, hx);
                float gh[5];
#pragma unroll
                for (int p = 0; p < 4; ++p) gh[p] = e32dot(*reinterpret_cast<const f4v(*)[4]>(&wr[4 * p]), hx);
                gh[4] = 0.0f;
                gh2_store(8 * (wave - 5), 4, gh);
                XSTAMPW(13, WRNN_XCD_STAMP_W13);
            }
        }
    step_end:
        XSTAMP_BAR();
        bar();
        // next step's x, GRU1 terms and the abort word: one LDS round trip
        const int ab = *abort_flag;
        const float xn = xs[t & 1];
        s4 = lds4(sg + 4 * tid);
        if (ab) return;
        if (wave != 0) x = xn;
    }
    // ---- carry the recurrent state to the next time chunk (every workgroup its own copy)
    __syncthreads();
    st[tid] = h1v;
    for (int i = tid; i < 4 * R; i += kXThreads) st[512 + i] = sg[i];
    if (tid < 48) st[512 + 2048 + tid] = gh2s[tid];
    if (li == 0) st[512 + 2048 + 48 + ui] = h2own;
    if (tid == 0) st[512 + 2048 + 48 + 16] = xs[(t_end - 1) & 1];
}

#define WRNN_K_XCD fatchord_xcd_kernel<false>
#define WRNN_K_XCD_DBG fatchord_xcd_kernel<true>

hipError_t launch_xcd(const XcdArgs &a, hipStream_t st) {
    XcdArgs args = a;
    void *params[] = {&args};
    const void *kf = a.dbg ? (const void *)WRNN_K_XCD_DBG : (const void *)WRNN_K_XCD;
    return hipLaunchKernel(kf, dim3(kXcds * kXcdWgs), dim3(kXThreads), params, xcd_lds_layout().total * sizeof(float), st);
}

hipError_t prepare_xcd_kernel(int max_lds_bytes) {
    for (const void *kf : {(const void *)WRNN_K_XCD, (const void *)WRNN_K_XCD_DBG}) {
        hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds_bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t xcd_occupancy(int *blocks_per_cu) {
    int best = 1 << 30;
    for (const void *kf : {(const void *)WRNN_K_XCD, (const void *)WRNN_K_XCD_DBG}) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kf, kXThreads, xcd_lds_layout().total * sizeof(float));
        if (e != hipSuccess) return e;
        best = n < best ? n : best;
    }
    *blocks_per_cu = best;
    return hipSuccess;
}

}  // namespace wrnn
