// fatchord_xcd2.hip — the XCD-resident MoL kernel of fatchord_xcd.hip (read its header first) with
// TWO rows per XCD: launch rows k and k + 8 on XCD k, up to 16 rows per launch.  It exists for the
// reference's default generation mode (hparams.py:58-60 voc_gen_batched, target 11000 / overlap
// 550: a 5 s utterance is 10 folds, models/fatchord_version.py:188-190) — 10 rows are two more
// than one per XCD, and the many-row MFMA kernel pays five hops and a quarter-used 4x4x1 MFMA at
// two rows per XCD.
//
// Same workgroup roles, hand-offs and LDS step flags as fatchord_xcd.hip; every per-row quantity
// is doubled and both rows move through each phase together, so a step still has three critical
// hops (Y, F1, F2) — each carries both rows' vectors (row r's granules kX2RowHop apart in the hop
// region) — and the weights held in VGPRs / LDS serve both rows:
//   GRU1: every thread evaluates its unit for both rows; GRU2: each engine's 3 dots against both
//   rows' h1; fc1 / fc2 waves poll both rows' y / f1 (8 × 16 B per lane) and run fc8_rows twice;
//   wave 0 polls both rows' 32 × 32 partial logits into its whole register set (it holds no
//   weights here: its W_hh2 rows 24..27 moved to LDS) and samples both rows.
// LDS for the second row's state (h1, h2, GRU1 terms, ring, …, ≈ 15 KB) comes from: W_hh1 rows
// 40..47 read from the slab (L2-resident, 16 KB per workgroup per step) by wave 7 instead of LDS,
// and a 3-step ring (xcd2_lds_layout: 163 760 of 163 840 bytes).
// Off the critical path as in fatchord_xcd.hip, for both rows: W_hh1·h1 → the GRU1 terms of step
// t + 1 (waves 0, 3, 4, 5, 7), the h2 gather (wave 6), S quarters (waves 1, 2, 5, 6), the ring
// (wave 7), W_hh2·h2 (LDS rows: waves 0, 1, 2; VGPR rows: waves 5..7).
// An XCD with one launch row runs the row twice (the copy's outputs and state are not written).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fatchord_loop.h"
#include "fatchord_xcd.h"
#include "wrnn_device.h"
#include "xcd_device.h"

namespace wrnn {

#define X2STAMPW(kk, w)                                                                                       \
    do {                                                                                                      \
        if (kDbg && a.dbg && wave == (w) && lane == 0 && t - a.t0 < a.dbg_steps)                              \
            a.dbg[((size_t)mem * a.dbg_steps + (t - a.t0)) * kStamps + (kk)] = (unsigned)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define X2STAMP(kk) X2STAMPW(kk, 0)

template <bool kDbg>
__global__ __launch_bounds__(kXThreads, 2) void fatchord_xcd2_kernel(XcdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int R = 512, TW = kXcdWgs * kXTerms, NR = kX2Rows;
    const Xcd2Lds ll = xcd2_lds_layout();
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 31, eng = lane >> 5;
    float *whh1 = smem + ll.whh1, *whh2l = smem + ll.whh2, *w3s = smem + ll.w3;
    float *ring = smem + ll.ring, *nzr = smem + ll.nz, *cst = smem + ll.cst, *xs = smem + ll.xs;
    auto H1S = [&](int r) { return smem + ll.h1 + r * 512; };
    auto H2S = [&](int r) { return smem + ll.h2 + r * 512; };
    auto SG = [&](int r) { return smem + ll.sg + r * 2048; };
    auto GH2S = [&](int r) { return smem + ll.gh2 + r * 48; };
    auto F2X = [&](int r) { return smem + ll.f2x + r * 32; };
    int *misc = reinterpret_cast<int *>(smem + ll.misc);
    int *abort_flag = misc, *h2ready = misc + 2, *f2ready = misc + 3, *ygot = misc + 4, *f1got = misc + 5;

    // ---- membership: XCD k (launch rows k, k + 8) and index c within it
    const int nx = min(a.nb, kXcds);   // XCDs with a row
    if (tid == 0) {
        const int k = (int)xcc_id();
        int c = kXcdWgs;
        if (k < nx) c = atomicAdd(&a.members[k], 1);
        misc[1] = (k < nx && c < kXcdWgs) ? k * kXcdWgs + c : -1;
        misc[0] = 0;
        for (int i = 2; i < 8; ++i) misc[i] = 0;
    }
    __syncthreads();
    const int mem = __builtin_amdgcn_readfirstlane(misc[1]);   // wave-uniform: hop addresses in SGPRs
    if (mem < 0) return;
    const int k = mem / kXcdWgs, c = mem - k * kXcdWgs;
    // launch row of this XCD's row r (a single-row XCD runs its row twice; the copy writes nothing)
    const bool valid1 = k + kXcds < a.nb;
    auto LROW = [&](int r) { return (r == 1 && valid1) ? k + kXcds : k; };
    const int t_end = a.t0 + a.Lc;
    const int t_terms = min(t_end, a.L - 1);
    unsigned long long *xg = a.xg + (size_t)k * kXXcdStride;
    auto XG = [&](int hop, int r) { return xg + (size_t)hop * kXHopStride + (size_t)r * kX2RowHop; };
    // the XCD's hop area as one buffer resource (SGPRs): publishes and row polls take 32-bit granule
    // indices instead of 64-bit addresses (fewer VGPRs live across the step loop)
    const __amdgpu_buffer_rsrc_t xgr = __builtin_amdgcn_make_buffer_rsrc(xg, 0, 0x7fffffff, 0x00020000);
    auto GI = [&](int hop, int r) { return hop * (int)kXHopStride + r * (int)kX2RowHop; };
    auto SLOT = [&](int t) { return t - kX2Ring * (t / kX2Ring); };
    auto RING = [&](int t, int r) { return ring + (SLOT(t) * NR + r) * kXTerms; };
    auto NZ = [&](int t, int r) { return nzr + (SLOT(t) * NR + r) * kXNoise; };
    auto TERMS = [&](int t, int r) {
        return a.terms + ((size_t)(t - a.t0) * a.nb + LROW(r)) * TW + (size_t)c * kXTerms;
    };
    const float *S = a.slab + (size_t)c * a.s.total;
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(S), 0, 0x7fffffff, 0x00020000);

    // ---- register-resident weights (as fatchord_xcd.hip; wave 0 holds none: wr is its F2 poll buffer)
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
        const int rb = 8 * (wave - 5);
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int m = 0; m < 4; ++m)
                wr[4 * p + m] = wave != 0 ? ldrow(S + a.s.whh2 + (rb + 2 * p + eng) * R, m) : f4v{0.0f, 0.0f, 0.0f, 0.0f};
    }
    const float q1r = S[a.s.q1a + tid], q1z = S[a.s.q1a + R + tid], q1n = S[a.s.q1a + 2 * R + tid];
    const int ui = wave * 2 + eng;
    const bool gh1w = wave == 0 || wave == 3 || wave == 4 || wave == 5 || wave == 7;
    const int gh0 = wave == 0 ? 0 : wave == 7 ? 40 : 10 * (wave - 2);
    auto noise_term = [&](int t, int r) -> float {
        float uu;
        if (a.noise) uu = a.noise[((size_t)t * a.Bt + a.b0 + LROW(r)) * 11 + lane];
        else uu = philox_noise(a.seed, (unsigned long long)(a.row0 + LROW(r)), (uint32_t)t, (uint32_t)lane, 1);
        return mol_noise_term(uu, lane);
    };
    auto publish_term = [&](int t, int r, int rr, float gh) {
        const int u = rr / 3, q = rr - 3 * u;
        const float p1 = RING(t, r)[XT_P1 + rr], bh = cst[XC_BHH1 + rr], bi = cst[XC_BIH1 + rr];
        const int g = GI(XH_S0 + (t & 1), r) + (c * kXUnits + u) * 4;
        const uint32_t tag = (uint32_t)t + 1u;
        if (q < 2) {
            xpub_b(xgr, g + q, tag, (gh + bh) + (p1 + bi));
        } else {
            xpub_b(xgr, g + 3, tag, gh + bh);
            xpub_b(xgr, g + 2, tag, p1 + bi);
        }
    };
    auto publish_terms = [&](int t, const float (&gh)[NR][5]) {
        const int rr = gh0 + 2 * li + eng;
        if (li < 5 && rr < 48) {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float v = li == 0 ? gh[r][0] : li == 1 ? gh[r][1] : li == 2 ? gh[r][2] : li == 3 ? gh[r][3] : gh[r][4];
                publish_term(t, r, rr, v);
            }
        }
    };
    // W_hh1·h1 for this wave's rows and both rows' h1: each weight row read once (LDS, or the slab
    // for rows ≥ kX2H1Lds: wave 7)
    auto gh1_dots = [&](float (&gh)[NR][5]) {
        f4v hx[NR][4];
#pragma unroll
        for (int r = 0; r < NR; ++r) e32x(H1S(r), li, hx[r]);
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            const int row = min(gh0 + 2 * p + eng, 47);
            f4v w4[4];
            if (wave == 7) {
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    w4[m] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(
                                                        srs, 4 * (a.s.whh1 + row * R + 4 * (li + 32 * m)), 0, 0));
            } else {
                e32x(whh1 + row * R, li, w4);
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) gh[r][p] = e32dot(w4, hx[r]);
        }
    };
    auto set_flag = [&](int *f, uint32_t tag) {
        if (lane == 0) __hip_atomic_store(f, (int)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto wait_flag = [&](int *f, uint32_t tag) {
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)tag)
            __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
    };
    auto gh2_store = [&](int r, int rb, int np, const float (&gh)[5]) {
        const int rr = rb + 2 * li + eng;
        if (li < np) GH2S(r)[rr] = li == 0 ? gh[0] : li == 1 ? gh[1] : li == 2 ? gh[2] : li == 3 ? gh[3] : gh[4];
    };
    // W_hh2·h2 of the LDS rows lr0 + 2p + e (p < np; LDS row index = W_hh2 row − kX2H2Lds0), both rows
    auto gh2_lds = [&](int lr0, int np) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            f4v hx[4];
            e32x(H2S(r), li, hx);
            float gh[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int p = 0; p < 5; ++p) {
                if (p < np) {
                    f4v w4[4];
                    e32x(whh2l + (lr0 - kX2H2Lds0 + 2 * p + eng) * R, li, w4);
                    gh[p] = e32dot(w4, hx);
                }
            }
            gh2_store(r, lr0, np, gh);
        }
    };
    auto gather_terms = [&](int t) {
        const int qq = wave <= 2 ? wave - 1 : wave - 3;
#pragma unroll
        for (int r = 0; r < NR; ++r)
            xgather16<4>(XG(XH_S0 + (t & 1), r) + qq * 512, (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t,
                         XH_S0 + (t & 1), abort_flag, lane, [&](int i, float v0, float v1) {
                             *reinterpret_cast<f2v *>(SG(r) + qq * 512 + i) = f2v{v0, v1};
                         });
    };
    // one row's 512 granules of a hop vector (pairs l + 64k) into v: loads issued by ld_row, the
    // tags checked (and re-polled, bounded) by poll_row — the next row's loads fly meanwhile
    auto ld_row = [&](int hop, int r, u4v (&v)[4]) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) v[kk] = ld16_sc1(xgr, 8 * GI(hop, r) + 16 * (lane + 64 * kk));
    };
    auto poll_row = [&](int hop, int r, uint32_t tag, int t, u4v (&v)[4]) {
        const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
        unsigned spins = 0;
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) ok &= (v[kk].y == tag) & (v[kk].w == tag);
            if (ok) return;
            ld_row(hop, r, v);
            if ((++spins & 63u) == 0) {
                const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (late || other) {
                    if (late) record_abort(a.ctl, -4, t, hop, blockIdx.x);
                    *abort_flag = 1;
                    return;
                }
            }
        }
    };

    // ---- prologue: W_hh1 rows 0..39 and W_hh2 rows 24..47 → LDS, fc3 columns, small vectors, ring
    // slots t0..t0+2 of both rows, state
    {
        const f4v *src = reinterpret_cast<const f4v *>(S + a.s.whh1);
        f4v *dst = reinterpret_cast<f4v *>(whh1);
        for (int i = tid; i < kX2H1Lds * R / 4; i += kXThreads) dst[i] = src[i];
        src = reinterpret_cast<const f4v *>(S + a.s.whh2 + kX2H2Lds0 * R);
        dst = reinterpret_cast<f4v *>(whh2l);
        for (int i = tid; i < (48 - kX2H2Lds0) * R / 4; i += kXThreads) dst[i] = src[i];
        for (int i = tid; i < kXFcRows * 32; i += kXThreads) w3s[i] = S[a.s.w3 + i];
        for (int i = tid; i < kXCst; i += kXThreads) cst[i] = S[a.s.cst + i];
        for (int t = a.t0; t < a.t0 + 3; ++t)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (t <= t_terms)
                    for (int i = tid; i < kXTerms; i += kXThreads) RING(t, r)[i] = TERMS(t, r)[i];
                if (wave == 1 && lane < 11 && t < a.L) NZ(t, r)[lane] = noise_term(t, r);
            }
    }
    const bool resume = a.t0 > 0;
    auto ST = [&](int r) { return a.state + ((size_t)(r == 1 ? k + kXcds : k) * kXcdWgs + c) * kXStateW; };
    float h1v[NR], h2own[NR], x[NR];
    f4v s4[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const float *st = ST(LROW(r) == k ? 0 : 1);
        h1v[r] = resume ? st[tid] : 0.0f;
        h2own[r] = resume ? st[512 + 2048 + 48 + ui] : 0.0f;
        if (resume) {
            for (int i = tid; i < 4 * R; i += kXThreads) SG(r)[i] = st[512 + i];
            if (tid < 48) GH2S(r)[tid] = st[512 + 2048 + tid];
            if (tid == 0) xs[2 * r + ((a.t0 + 1) & 1)] = st[512 + 2048 + 48 + 16];
        } else {
            if (tid < 48) GH2S(r)[tid] = 0.0f;
            if (tid == 0) xs[2 * r + 1] = 0.0f;
        }
    }
    __syncthreads();
    if (!resume) {   // GRU1 terms of step 0 (GH1 = 0), published and gathered
        if (gh1w) {
            const float z5[NR][5] = {};
            publish_terms(0, z5);
        }
        if (wave == 1 || wave == 2 || wave == 5 || wave == 6) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            gather_terms(0);
        }
    }
    __syncthreads();
    if (*abort_flag) return;

#pragma unroll
    for (int r = 0; r < NR; ++r) {
        x[r] = xs[2 * r + ((a.t0 + 1) & 1)];
        s4[r] = lds4(SG(r) + 4 * tid);
    }
    for (int t = a.t0; t < t_end; ++t) {
        const uint32_t tag = (uint32_t)t + 1u;
        const bool more = t + 1 < a.L;
        X2STAMP(0);
        float p2q[NR][3], xi[NR], ghv[NR][3];
        {
            float q2v[3], bi2[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                q2v[q] = cst[XC_Q2 + ui * 3 + q];
                bi2[q] = cst[XC_BIH2 + ui * 3 + q];
            }
            const float wi0v = cst[XC_WI0 + ui];
            // ---- GRU1 (:208-210), unit tid, both rows
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float *tr = RING(t, r);
#pragma unroll
                for (int q = 0; q < 3; ++q) ghv[r][q] = GH2S(r)[ui * 3 + q] + cst[XC_BHH2 + ui * 3 + q];
                const float rg = sigmoid_(fmaf(x[r], q1r, s4[r].x));
                const float zg = sigmoid_(fmaf(x[r], q1z, s4[r].y));
                const float ng = tanh_(fmaf(x[r], q1n, s4[r].z) + s4[r].w * rg);
                h1v[r] = (h1v[r] - ng) * zg + ng;
                H1S(r)[tid] = h1v[r];
#pragma unroll
                for (int q = 0; q < 3; ++q) p2q[r][q] = fmaf(x[r], q2v[q], tr[XT_P2 + ui * 3 + q]) + bi2[q];
                xi[r] = fmaf(wi0v, x[r], tr[XT_CI + ui]);
            }
        }
        bar();
        X2STAMP(1);
        // ---- GRU2 (:212-214), both rows: engine ui's 3 gate rows against each row's h1
        {   // both rows' dots first, then both gate chains, then both publishes (one window)
            float g[NR][3], yv[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                f4v hx[4];
                e32x(H1S(r), li, hx);
#pragma unroll
                for (int q = 0; q < 3; ++q) g[r][q] = e32dot(wih2[q], hx);
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float h1j = H1S(r)[c * kXUnits + ui];
                const float hn = gru_gate_math(g[r][0] + p2q[r][0], g[r][1] + p2q[r][1], g[r][2] + p2q[r][2], ghv[r][0],
                                               ghv[r][1], ghv[r][2], h2own[r]);
                h2own[r] = hn;
                yv[r] = (xi[r] + h1j) + hn;
            }
            if (li == 0) {
#pragma unroll
                for (int r = 0; r < NR; ++r) xpub_b(xgr, GI(XH_Y, r) + c * kXUnits + ui, tag, yv[r]);
            }
        }
        X2STAMP(2);
        auto pub_h2 = [&]() {
            if (li == 0) {
#pragma unroll
                for (int r = 0; r < NR; ++r) xpub_b(xgr, GI(XH_H2, r) + c * kXUnits + ui, tag, h2own[r]);
            }
        };
        const int jq = lane & 1, rho = jq + 2 * (lane >> 4);
        if (wave == 0) {
            if (more) {
                float gh[NR][5];
                gh1_dots(gh);
                wait_flag(ygot, tag);
                publish_terms(t + 1, gh);
                pub_h2();
            }
            // ---- hop F2, both rows: Σ of the 32 workgroups' partials + b3 → sample
            const int jp = lane & 15, pg = lane >> 4;
            float ua[NR], ub[NR], u10[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                ua[r] = NZ(t, r)[jp < 5 ? 2 * jp : 0];
                ub[r] = NZ(t, r)[jp < 5 ? 2 * jp + 1 : 0];
                u10[r] = NZ(t, r)[10];
            }
            const float b3a = cst[XC_B3 + 2 * jp], b3b = cst[XC_B3 + 2 * jp + 1];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int goff = pg * 8 * kXF2Line * 8 + jp * 16;
            // row r's 32 × 32 partials: lane l's eight 16-byte loads (logits 2jp, 2jp + 1 of producers
            // 8·(l >> 4) + m) into wr[8r .. 8r + 7]; row 1's loads fly while row 0 is summed and sampled
            u4v *v = reinterpret_cast<u4v *>(&wr[0]);   // wave 0 holds no weights here
            auto ld_f2 = [&](int r) {
#pragma unroll
                for (int m = 0; m < 8; ++m) v[8 * r + m] = ld16_sc1(xgr, 8 * GI(XH_F2, r) + goff + m * kXF2Line * 8);
            };
            auto poll_f2 = [&](int r) {
                const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
                unsigned spins = 0;
                for (;;) {
                    bool ok = true;
#pragma unroll
                    for (int m = 0; m < 8; ++m) ok &= (v[8 * r + m].y == tag) & (v[8 * r + m].w == tag);
                    if (ok) return;
                    ld_f2(r);
                    if ((++spins & 63u) == 0) {
                        const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                        const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                        if (late || other) {
                            if (late) record_abort(a.ctl, -4, t, XH_F2, blockIdx.x);
                            *abort_flag = 1;
#pragma unroll
                            for (int m = 0; m < 8; ++m) v[8 * r + m] = u4v{0u, tag, 0u, tag};
                            return;
                        }
                    }
                }
            };
            ld_f2(0);
            ld_f2(1);
            poll_f2(0);
            X2STAMP(7);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (r > 0) poll_f2(r);
                float pa[8], pb[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    pa[m] = __uint_as_float(v[8 * r + m].x);
                    pb[m] = __uint_as_float(v[8 * r + m].z);
                }
#pragma unroll
                for (int n = 4; n >= 1; n /= 2)
#pragma unroll
                    for (int m = 0; m < n; ++m) {
                        pa[m] += pa[m + n];
                        pb[m] += pb[m + n];
                    }
                const float la = cross_rows(pa[0]) + b3a, lb = cross_rows(pb[0]) + b3b;
                x[r] = mol_sample_pairs(la, lb, ua[r], ub[r], u10[r], jp);
            }
            if (lane == 0) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    xs[2 * r + (t & 1)] = x[r];
                    if (c == 0 && (r == 0 || valid1)) a.out[(size_t)(a.b0 + LROW(r)) * a.L + t] = x[r];
                }
            }
            X2STAMP(8);
        } else if (wave < kXWaveFc2) {
            // ---- hop Y (both rows) → fc1 rows 8h.. → relu → hop F1
            const int hf = wave - kXWaveFc1, rg = 8 * hf + rho;
            float v1[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) v1[r] = RING(t, r)[XT_V1 + rg];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u4v v[NR][4];
#pragma unroll
            for (int r = 0; r < NR; ++r) ld_row(XH_Y, r, v[r]);
#pragma unroll
            for (int r = 0; r < NR; ++r) poll_row(XH_Y, r, tag, t, v[r]);
            if (hf == 0) set_flag(ygot, tag);
            X2STAMPW(3, 1);
            float A[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                f2v yk[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) yk[kk] = f2v{__uint_as_float(v[r][kk].x), __uint_as_float(v[r][kk].z)};
                float o[2];
                fc8_rows(wr, yk, o);
                A[r] = (jq == 0 ? o[0] : o[1]) + v1[r];
            }
            if ((lane & 15) < 2) {
#pragma unroll
                for (int r = 0; r < NR; ++r)
                    xpub_b(xgr, GI(XH_F1, r) + c * kXFcRows + rg, tag, A[r] > 0.0f ? A[r] : 0.0f);
            }
            X2STAMPW(4, 1);
            if (more) {   // h2 out; after f1 gathered: a quarter of the next S; W_hh2 LDS rows 28 + 10h + 2p + e
                pub_h2();
                wait_flag(f1got, tag);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                gather_terms(t + 1);
                wait_flag(h2ready, tag);
                gh2_lds(28 + 10 * hf, 5);
                X2STAMPW(11, 1);
            }
        } else if (wave < kXWaveFc2 + 2) {
            const int hf = wave - kXWaveFc2;
            if (more) {   // W_hh1 rows; after y gathered their terms and h2 out
                float gh[NR][5];
                gh1_dots(gh);
                wait_flag(ygot, tag);
                publish_terms(t + 1, gh);
                pub_h2();
            }
            X2STAMPW(9, 3);
            // ---- hop F1 (both rows) → fc2 rows 8h.. → relu → fc3 partial logits; wave 4 hands its
            // partials to wave 3 (LDS flag), wave 3 publishes both rows' lines (hop F2)
            float v2[NR][2], w3c[8];
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
                for (int j = 0; j < 2; ++j) v2[r][j] = RING(t, r)[XT_V2 + 8 * hf + j + 2 * (lane >> 4)];
#pragma unroll
            for (int r = 0; r < 8; ++r) w3c[r] = w3s[(8 * hf + r) * 32 + li];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u4v v[NR][4];
#pragma unroll
            for (int r = 0; r < NR; ++r) ld_row(XH_F1, r, v[r]);
#pragma unroll
            for (int r = 0; r < NR; ++r) poll_row(XH_F1, r, tag, t, v[r]);
            if (hf == 0) set_flag(f1got, tag);
            X2STAMPW(5, 3);
            float p[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                f2v fk[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) fk[kk] = f2v{__uint_as_float(v[r][kk].x), __uint_as_float(v[r][kk].z)};
                float o[2];
                fc8_rows(wr, fk, o);
                p[r] = 0.0f;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const float f = o[j] + v2[r][j];
                    const float f2 = f > 0.0f ? f : 0.0f;
#pragma unroll
                    for (int g = 0; g < 4; ++g) p[r] = fmaf(w3c[j + 2 * g], lane_bcast(f2, 16 * g), p[r]);
                }
            }
            if (hf == 1) {
                if (lane < 32) {
#pragma unroll
                    for (int r = 0; r < NR; ++r) F2X(r)[lane] = p[r];
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                set_flag(f2ready, tag);
            } else {
                unsigned spin = 0;
                while (__hip_atomic_load(f2ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)tag) {
                    if ((++spin & 255u) == 0 &&
                        __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                        break;
                }
                asm volatile("" ::: "memory");
                if (lane < kXF2Line) {
#pragma unroll
                    for (int r = 0; r < NR; ++r) xpub_b(xgr, GI(XH_F2, r) + c * kXF2Line + lane, tag, p[r] + F2X(r)[lane]);
                }
                X2STAMPW(6, 3);
            }
            if (more) {   // W_hh2·h2 of the LDS rows 24 + 2hf + e (after their F2 duty: off wave 0's path)
                wait_flag(h2ready, tag);
                gh2_lds(24 + 2 * hf, 1);
            }
        } else if (more) {
            // ---- waves 5..7: W_hh1 rows (5; 7 from the slab) → after y gathered their terms and h2
            // out; after f1 gathered: h2 (wave 6, then flag), S quarters (5, 6), the ring (7); after
            // h2 gathered: W_hh2·h2 (VGPR rows)
            if (wave != 6) {
                float gh[NR][5];
                gh1_dots(gh);
                wait_flag(ygot, tag);
                publish_terms(t + 1, gh);
            } else {
                wait_flag(ygot, tag);
            }
            pub_h2();
            wait_flag(f1got, tag);
            if (wave == 6) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int r = 0; r < NR; ++r)
                    xgather16<4>(XG(XH_H2, r), tag, a.ctl, a.timeout_ticks, t, XH_H2, abort_flag, lane,
                                 [&](int i, float v0, float v1) { *reinterpret_cast<f2v *>(H2S(r) + i) = f2v{v0, v1}; });
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                set_flag(h2ready, tag);
                X2STAMPW(10, 6);
            }
            if (wave <= 6) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                gather_terms(t + 1);
                X2STAMPW(14, 5);
            } else if (t + 2 >= a.t0 + 3) {
                // ring: step t+2's terms and sampler noise of both rows
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    if (t + 2 <= t_terms && lane < kXTerms / 4)
                        reinterpret_cast<f4v *>(RING(t + 2, r))[lane] = reinterpret_cast<const f4v *>(TERMS(t + 2, r))[lane];
                    if (t + 2 < a.L && lane < 11) NZ(t + 2, r)[lane] = noise_term(t + 2, r);
                }
                X2STAMPW(12, 7);
            }
            wait_flag(h2ready, tag);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                f4v hx[4];
                e32x(H2S(r), li, hx);
                float gh[5];
#pragma unroll
                for (int p = 0; p < 4; ++p) gh[p] = e32dot(*reinterpret_cast<const f4v(*)[4]>(&wr[4 * p]), hx);
                gh[4] = 0.0f;
                gh2_store(r, 8 * (wave - 5), 4, gh);
            }
            X2STAMPW(13, 5);
        }
        bar();
        const int ab = *abort_flag;
        float xn[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            xn[r] = xs[2 * r + (t & 1)];
            s4[r] = lds4(SG(r) + 4 * tid);
        }
        if (ab) return;
        if (wave != 0) {
#pragma unroll
            for (int r = 0; r < NR; ++r) x[r] = xn[r];
        }
    }
    // ---- carry both rows' recurrent state to the next time chunk (the copy row of a single-row XCD
    // writes nothing)
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        if (r == 1 && !valid1) break;
        float *st = ST(r);
        st[tid] = h1v[r];
        for (int i = tid; i < 4 * R; i += kXThreads) st[512 + i] = SG(r)[i];
        if (tid < 48) st[512 + 2048 + tid] = GH2S(r)[tid];
        if (li == 0) st[512 + 2048 + 48 + ui] = h2own[r];
        if (tid == 0) st[512 + 2048 + 48 + 16] = xs[2 * r + ((t_end - 1) & 1)];
    }
}

hipError_t launch_xcd2(const XcdArgs &a, hipStream_t st) {
    XcdArgs args = a;
    void *params[] = {&args};
    const void *kf = a.dbg ? (const void *)fatchord_xcd2_kernel<true> : (const void *)fatchord_xcd2_kernel<false>;
    return hipLaunchKernel(kf, dim3(kXcds * kXcdWgs), dim3(kXThreads), params, xcd2_lds_layout().total * sizeof(float),
                           st);
}

hipError_t prepare_xcd2_kernel(int max_lds_bytes) {
    for (const void *kf : {(const void *)fatchord_xcd2_kernel<false>, (const void *)fatchord_xcd2_kernel<true>}) {
        hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds_bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t xcd2_occupancy(int *blocks_per_cu) {
    int best = 1 << 30;
    for (const void *kf : {(const void *)fatchord_xcd2_kernel<false>, (const void *)fatchord_xcd2_kernel<true>}) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kf, kXThreads, xcd2_lds_layout().total * sizeof(float));
        if (e != hipSuccess) return e;
        best = n < best ? n : best;
    }
    *blocks_per_cu = best;
    return hipSuccess;
}

}  // namespace wrnn
