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
// GRU2, gather S (waves 5, 6), LDS-DMA of the conditioning terms and noise (wave 7).
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

namespace wrnn {

__device__ __forceinline__ unsigned xcc_id() {
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xF;   // HW_REG_XCC_ID[3:0]
}

// XCD-local publish: a plain (workgroup-scope) 8-byte store keeps the line in this XCD's L2
__device__ __forceinline__ void xpub(unsigned long long *g, uint32_t tag, float v) {
    const unsigned long long x = ((unsigned long long)tag << 32) | __float_as_uint(v);
    __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ float perm_sum16(float v) {   // + the same lane of the paired 16-lane row
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float perm_sum32(float v) {   // + the same lane of the other wave half
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
// Σ over the 4 DPP rows of a wave (identical bits in the lanes it pairs)
__device__ __forceinline__ float cross_rows(float v) { return perm_sum32(perm_sum16(v)); }

// Wave-wide dot partials of NR rows held in registers (lane l: chunks 4l and 256 + 4l) against
// x (LDS, natural order): p[r] = this lane's 8 products, packed FMAs.
template <int NR>
__device__ __forceinline__ void wdot(const f4v (&w)[NR][2], const f4v (&x)[2], float *p) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        f2v a = __builtin_elementwise_fma(w[r][0].xy, x[0].xy, f2v{0.0f, 0.0f});
        f2v b = __builtin_elementwise_fma(w[r][1].xy, x[1].xy, f2v{0.0f, 0.0f});
        a = __builtin_elementwise_fma(w[r][0].zw, x[0].zw, a);
        b = __builtin_elementwise_fma(w[r][1].zw, x[1].zw, b);
        const f2v s = a + b;
        p[r] = s.x + s.y;
    }
}

// 8 per-lane partials → wave totals: lane l returns A = Σ p[l & 3], B = Σ p[4 + (l & 3)]
__device__ __forceinline__ void reduce8(const float (&p)[8], int lane, float &A, float &B) {
    const float a4[4] = {p[0], p[1], p[2], p[3]}, b4[4] = {p[4], p[5], p[6], p[7]};
    A = cross_rows(row_reduce_scatter4(a4, lane));
    B = cross_rows(row_reduce_scatter4(b4, lane));
}

__device__ __forceinline__ f4v lds4(const float *p) { return *reinterpret_cast<const f4v *>(p); }

// Poll NG granules per lane (indices lid + 64·k: one address per call site, instruction
// immediates for k) until all carry `tag`, then store(i, value).  Bounded like wrnn_device.h:gather (timeout / another workgroup's abort).
template <int NG, typename Store>
__device__ __forceinline__ void xgather(const unsigned long long *g, uint32_t tag, int *ctl, long long timeout,
                                        int step, int hop, int *lds_abort, int lid, Store store) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (;;) {
        unsigned long long v[NG];
#pragma unroll
        for (int k = 0; k < NG; ++k) v[k] = __hip_atomic_load(g + lid + 64 * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int k = 0; k < NG; ++k) ok &= (uint32_t)(v[k] >> 32) == tag;
        if (ok) {
#pragma unroll
            for (int k = 0; k < NG; ++k) store(lid + 64 * k, __uint_as_float((uint32_t)v[k]));
            return;
        }
        if ((++spins & 63u) == 0) {
            const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout;
            const bool other = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (late || other) {
                if (late) record_abort(ctl, -4, step, hop, blockIdx.x);
                *lds_abort = 1;
                return;
            }
        }
    }
}

#define XSTAMP(kk)                                                                                            \
    do {                                                                                                      \
        if (kDbg && a.dbg && tid == 0 && t - a.t0 < a.dbg_steps)                                              \
            a.dbg[((size_t)mem * a.dbg_steps + (t - a.t0)) * kStamps + (kk)] = (unsigned)__builtin_amdgcn_s_memrealtime(); \
    } while (0)

template <bool kDbg>
__global__ __launch_bounds__(kXThreads, 2) void fatchord_xcd_kernel(XcdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int R = 512, NC = 30, TW = kXcdWgs * kXTerms;
    const XcdLds ll = xcd_lds_layout();
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float *whh1 = smem + ll.whh1, *whh2l = smem + ll.whh2, *h1s = smem + ll.h1, *ys = smem + ll.y;
    float *f1s = smem + ll.f1, *h2s = smem + ll.h2, *sg = smem + ll.sg, *part = smem + ll.part;
    float *ring = smem + ll.ring, *nzr = smem + ll.nz, *gh2s = smem + ll.gh2, *cst = smem + ll.cst, *xs = smem + ll.xs;
    int *misc = reinterpret_cast<int *>(smem + ll.misc);
    int *abort_flag = misc;

    // ---- membership: XCD k (row b0 + k) and index c within it
    if (tid == 0) {
        const int k = (int)xcc_id();
        int c = kXcdWgs;
        if (k < a.nb) c = atomicAdd(&a.members[k], 1);
        misc[1] = (k < a.nb && c < kXcdWgs) ? k * kXcdWgs + c : -1;
        misc[0] = 0;
    }
    __syncthreads();
    const int mem = misc[1];
    if (mem < 0) return;
    const int k = mem / kXcdWgs, c = mem - k * kXcdWgs;
    const int b = a.b0 + k;
    const int t_end = a.t0 + a.Lc;
    const int t_terms = min(t_end, a.L - 1);
    unsigned long long *xg = a.xg + (size_t)k * kXXcdStride;
    auto XG = [&](int hop) { return xg + (size_t)hop * kXHopStride; };
    auto RING = [&](int t) { return ring + (t & (kXRing - 1)) * kXTerms; };
    auto NZ = [&](int t) { return nzr + (t & (kXRing - 1)) * kXNoise; };
    auto TERMS = [&](int t) { return a.terms + ((size_t)(t - a.t0) * a.nb + k) * TW + (size_t)c * kXTerms; };
    const float *S = a.slab + (size_t)c * a.s.total;
    const unsigned long long prow = (unsigned long long)(a.row0 + k);

    // ---- register-resident weights (lane l: chunks 4l and 256 + 4l of every row)
    f4v wih2[6][2], w1r[2][2], w2r[2][2], whh2r[kXH2Reg][2];
    auto ldrow = [&](const float *row, int h) { return *reinterpret_cast<const f4v *>(row + 4 * lane + 256 * h); };
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int r = 0; r < 6; ++r) wih2[r][h] = ldrow(S + a.s.wih2 + (wave * 6 + r) * R, h);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            w1r[r][h] = ldrow(S + a.s.w1 + (wave * 2 + r) * R, h);
            w2r[r][h] = ldrow(S + a.s.w2 + (wave * 2 + r) * R, h);
        }
#pragma unroll
        for (int r = 0; r < kXH2Reg; ++r)
            whh2r[r][h] = wave >= 1 ? ldrow(S + a.s.whh2 + ((wave - 1) * kXH2Reg + r) * R, h) : f4v{0.0f, 0.0f, 0.0f, 0.0f};
    }
    const float w3a = S[a.s.w3 + (wave * 2 + 0) * 32 + (lane & 31)];
    const float w3b = S[a.s.w3 + (wave * 2 + 1) * 32 + (lane & 31)];
    // GRU1 of unit tid: x-coefficients
    const float q1r = S[a.s.q1a + tid], q1z = S[a.s.q1a + R + tid], q1n = S[a.s.q1a + 2 * R + tid];
    const int ui = wave * 2 + (lane & 1);            // lanes 0/1: local unit (and fc row) 2·wave + i
    // W_hh1 rows of this wave (waves 1..7): gh0 + r, r < 7; lane l < 8 owns row gh0 + (l < 4 ? l : 4 + (l & 3))
    const int gh0 = (wave - 1) * kXGhRows;
    const int rr = gh0 + (lane < 4 ? lane : 4 + (lane & 3));
    const bool rr_ok = wave >= 1 && lane < 8 && (lane < 4 || (lane & 3) < kXGhRows - 4) && rr < 48;
    // W_hh2 rows of this wave: kXH2Reg in VGPRs (rows (w-1)·4 + r), 3 from LDS (rows 28 + (w-1)·3 + r)
    const int h2l0 = (wave - 1) * 3;
    const int rr2 = lane < 4 ? (wave - 1) * kXH2Reg + lane : kXH2RegRows + h2l0 + (lane & 3);
    const bool rr2_ok = wave >= 1 && lane < 8 && (lane < 4 || ((lane & 3) < 3 && rr2 < 48));

    // sampler noise of step t → NZ(t): u1 → log(-log u1) (distribution.py:107), u2 → log u2 − log(1 − u2) (:119)
    auto noise_term = [&](int t) -> float {
        float uu;
        if (a.noise) uu = a.noise[((size_t)t * a.Bt + b) * 11 + lane];
        else uu = philox_noise(a.seed, prow, (uint32_t)t, (uint32_t)lane, 1);
        return mol_noise_term(uu, lane);
    };
    // GRU1 terms of step t for this wave's W_hh1 rows (lane-parallel, rows rr):
    //   q = 0: S_r = (GH1_r + b_hh,r) + (P1_r + b_ih,r), q = 1: S_z likewise,
    //   q = 2: Gh_n = GH1_n + b_hh,n (term 3) and Gi_n = P1_n + b_ih,n (term 2)
    auto publish_terms = [&](int t, float gh) {
        if (!rr_ok) return;
        const int u = rr / 3, q = rr - 3 * u;
        const float p1 = RING(t)[XT_P1 + rr], bh = cst[XC_BHH1 + rr], bi = cst[XC_BIH1 + rr];
        unsigned long long *g = XG(XH_S0 + (t & 1)) + (size_t)(c * kXUnits + u) * 4;
        const uint32_t tag = (uint32_t)t + 1u;
        if (q < 2) {
            xpub(g + q, tag, (gh + bh) + (p1 + bi));
        } else {
            xpub(g + 3, tag, gh + bh);
            xpub(g + 2, tag, p1 + bi);
        }
    };
    // gather half of step t's GRU1 terms (waves 5 and 6: 1024 granules each, two chunks of 512)
    auto gather_terms = [&](int t) {
        const int half = wave - 5;
        for (int c0 = 0; c0 < 1024; c0 += 512) {
            xgather<8>(XG(XH_S0 + (t & 1)) + half * 1024 + c0, (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t,
                       XH_S0 + (t & 1), abort_flag, lane, [&](int i, float v) { sg[half * 1024 + c0 + i] = v; });
            if (*reinterpret_cast<volatile int *>(abort_flag)) return;
        }
    };

    // ---- prologue: W_hh1 and the LDS rows of W_hh2, small vectors, ring slots t0..t0+2, state
    {
        const f4v *src = reinterpret_cast<const f4v *>(S + a.s.whh1);
        f4v *dst = reinterpret_cast<f4v *>(whh1);
        for (int i = tid; i < 48 * R / 4; i += kXThreads) dst[i] = src[i];
        src = reinterpret_cast<const f4v *>(S + a.s.whh2 + kXH2RegRows * R);
        dst = reinterpret_cast<f4v *>(whh2l);
        for (int i = tid; i < (48 - kXH2RegRows) * R / 4; i += kXThreads) dst[i] = src[i];
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
    float h2own = resume ? st[512 + 2048 + 48 + ui] : 0.0f;   // h2 of this lane's own unit
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
        publish_terms(0, 0.0f);
        if (wave == 5 || wave == 6) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            gather_terms(0);
        }
    }
    __syncthreads();
    if (*abort_flag) return;

    float x = xs[(a.t0 + 1) & 1];    // x_{t-1}, wave-uniform
    f4v pre_terms = {0.0f, 0.0f, 0.0f, 0.0f};   // wave 7: step t+3's terms / raw noise in flight
    float pre_noise = 0.5f;
    for (int t = a.t0; t < t_end; ++t) {
        const uint32_t tag = (uint32_t)t + 1u;
        const bool more = t + 1 < a.L;
        const float *tr = RING(t);
        XSTAMP(0);
        // ---- GRU1 (:208-210), unit tid
        {
            const f4v s4 = lds4(sg + 4 * tid);
            const float r = sigmoid_(fmaf(x, q1r, s4.x));
            const float z = sigmoid_(fmaf(x, q1z, s4.y));
            const float n = tanh_(fmaf(x, q1n, s4.z) + s4.w * r);
            h1v = (h1v - n) * z + n;
            h1s[tid] = h1v;
        }
        // operands of the GRU2 gate math (lanes 0/1: unit ui), issued before the barrier
        float p2q[3], ghv[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            p2q[q] = fmaf(x, cst[XC_Q2 + ui * 3 + q], tr[XT_P2 + ui * 3 + q]);
            ghv[q] = gh2s[ui * 3 + q] + cst[XC_BHH2 + ui * 3 + q];
        }
        const float xi = fmaf(cst[XC_WI0 + ui], x, tr[XT_CI + ui]);   // x_I of unit ui
        bar();
        XSTAMP(1);
        // ---- GRU2 (:212-214): W_ih2[:, :R]·h1 for rows (gate q, unit i) = 2q + i
        {
            const f4v hx[2] = {lds4(h1s + 4 * lane), lds4(h1s + 256 + 4 * lane)};
            const float h1j = h1s[c * kXUnits + ui];
            float p[8];
            wdot<6>(wih2, hx, p);
            p[6] = p[7] = 0.0f;
            float A, B;
            reduce8(p, lane, A, B);
            // lane i (0/1): gate r = A (row i), z = A of lane i + 2 (row 2 + i), n = B (row 4 + i)
            const float Az = WRNN_DPP(A, 0x4E);      // quad_perm [2,3,0,1]
            const float gi_r = (A + p2q[0]) + cst[XC_BIH2 + ui * 3 + 0];
            const float gi_z = (Az + p2q[1]) + cst[XC_BIH2 + ui * 3 + 1];
            const float gi_n = (B + p2q[2]) + cst[XC_BIH2 + ui * 3 + 2];
            const float hn = gru_gate_math(gi_r, gi_z, gi_n, ghv[0], ghv[1], ghv[2], h2own);
            h2own = hn;
            // y = (x_I + h1) + h2 (:212, :216)
            const float y = (xi + h1j) + hn;
            if (lane < 2) {
                xpub(XG(XH_Y) + c * kXUnits + ui, tag, y);
                xpub(XG(XH_H2) + c * kXUnits + ui, tag, hn);
            }
        }
        XSTAMP(2);
        // ---- hop Y (wave 0) ‖ W_hh1·h1 → GRU1 terms of step t+1 (waves 1..7)
        if (wave == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            xgather<8>(XG(XH_Y), tag, a.ctl, a.timeout_ticks, t, XH_Y, abort_flag, lane, [&](int i, float v) { ys[i] = v; });
            XSTAMP(3);
        } else if (more) {
            const f4v hx[2] = {lds4(h1s + 4 * lane), lds4(h1s + 256 + 4 * lane)};
            float p[8];
            const float *wb = whh1 + gh0 * R + 4 * lane;   // wave 7's 7th row (48) reads past W_hh1: unused
#pragma unroll
            for (int r = 0; r < kXGhRows; ++r) {   // W_hh1 rows streamed from LDS
                const f4v wr[1][2] = {{lds4(wb + r * R), lds4(wb + r * R + 256)}};
                wdot<1>(wr, hx, p + r);
            }
            p[7] = 0.0f;
            float A, B;
            reduce8(p, lane, A, B);
            publish_terms(t + 1, lane < 4 ? A : B);
        }
        const float v1 = tr[XT_V1 + ui], v2 = tr[XT_V2 + ui];
        bar();
        // ---- fc1 (:216-218), rows 2w + i → relu → hop F1
        {
            const f4v yx[2] = {lds4(ys + 4 * lane), lds4(ys + 256 + 4 * lane)};
            float p[4];
            wdot<2>(w1r, yx, p);
            p[2] = p[3] = 0.0f;
            const float A = cross_rows(row_reduce_scatter4(p, lane)) + v1;
            if (lane < 2) xpub(XG(XH_F1) + c * kXFcRows + ui, tag, A > 0.0f ? A : 0.0f);
        }
        XSTAMP(4);
        if (wave == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            xgather<8>(XG(XH_F1), tag, a.ctl, a.timeout_ticks, t, XH_F1, abort_flag, lane, [&](int i, float v) { f1s[i] = v; });
            XSTAMP(5);
        } else if (wave == 6 && more) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            xgather<8>(XG(XH_H2), tag, a.ctl, a.timeout_ticks, t, XH_H2, abort_flag, lane, [&](int i, float v) { h2s[i] = v; });
        }
        bar();
        // ---- fc2 (:220-221) → relu → fc3 partial logits of the 16 own f2 rows (:223)
        {
            const f4v fx[2] = {lds4(f1s + 4 * lane), lds4(f1s + 256 + 4 * lane)};
            float p[4];
            wdot<2>(w2r, fx, p);
            p[2] = p[3] = 0.0f;
            float A = cross_rows(row_reduce_scatter4(p, lane)) + v2;
            A = A > 0.0f ? A : 0.0f;
            const float f20 = lane_bcast(A, 0), f21 = lane_bcast(A, 1);
            if (lane < 32) part[wave * 32 + lane] = fmaf(w3b, f21, w3a * f20);
        }
        bar();
        XSTAMP(6);
        if (wave == 0) {
            // Σ of the 8 waves' partials → hop F2 → Σ of the 32 workgroups' partials + b3 → sample
            if (lane < NC) {
                float s = 0.0f;
#pragma unroll
                for (int w = 0; w < kXWaves; ++w) s += part[w * 32 + lane];
                xpub(XG(XH_F2) + c * kXF2Line + lane, tag, s);
            }
            const float ul = NZ(t)[lane < 10 ? lane : 0], u10 = NZ(t)[10], b3v = cst[XC_B3 + (lane & 31)];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // lane l: logit j = l & 31 of producers 16·(l >> 5) + m, m = 0..15 (256 B apart: immediates)
            const int j = lane & 31, jj = j < NC ? j : 0;
            const unsigned long long *gp = XG(XH_F2);
            const unsigned long long *gl = gp + (lane >> 5) * 16 * kXF2Line + jj;
            const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
            unsigned spins = 0;
            float pv[16];
            for (;;) {
                unsigned long long v[16];
#pragma unroll
                for (int m = 0; m < 16; ++m)
                    v[m] = __hip_atomic_load(gl + m * kXF2Line, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                bool ok = true;
#pragma unroll
                for (int m = 0; m < 16; ++m) ok &= (uint32_t)(v[m] >> 32) == tag;
                if (ok) {
#pragma unroll
                    for (int m = 0; m < 16; ++m) pv[m] = __uint_as_float((uint32_t)v[m]);
                    break;
                }
                if ((++spins & 63u) == 0) {
                    const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                    const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    if (late || other) {
                        if (late) record_abort(a.ctl, -4, t, XH_F2, blockIdx.x);
                        *abort_flag = 1;
#pragma unroll
                        for (int m = 0; m < 16; ++m) pv[m] = 0.0f;
                        break;
                    }
                }
            }
            XSTAMP(7);
#pragma unroll
            for (int n = 8; n >= 1; n /= 2)
#pragma unroll
                for (int m = 0; m < n; ++m) pv[m] += pv[m + n];
            const float s = perm_sum32(pv[0]) + b3v;
            x = mol_sample_reg(s, ul, u10, lane);
            if (lane == 0) {
                xs[t & 1] = x;
                if (c == 0) a.out[(size_t)b * a.L + t] = x;
            }
            XSTAMP(8);
        } else if (more) {
            // W_hh2·h2 (h2 gathered by wave 6 before the barrier) → gh2s for the next GRU2
            const f4v hx[2] = {lds4(h2s + 4 * lane), lds4(h2s + 256 + 4 * lane)};
            float p[8];
            wdot<kXH2Reg>(whh2r, hx, p);
            const float *wb = whh2l + h2l0 * R + 4 * lane;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                // wave 7 has two LDS rows (18, 19): its third pass re-reads row 19 (result unused)
                const int ro = (r == 2 && wave == 7) ? R : r * R;
                const f4v wr[1][2] = {{lds4(wb + ro), lds4(wb + ro + 256)}};
                wdot<1>(wr, hx, p + kXH2Reg + r);
            }
            p[7] = 0.0f;
            float A, B;
            reduce8(p, lane, A, B);
            if (rr2_ok) gh2s[rr2] = lane < 4 ? A : B;
            if (wave == 5 || wave == 6) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                gather_terms(t + 1);
            }
            if (wave == 7) {
                // ring: step t+2's terms and raw noise, loaded into registers at step t-1, into LDS;
                // then the loads of step t+3 (registers, not LDS-DMA: hipcc waits for an LDS-DMA
                // before every later LDS access of the issuing wave)
                if (t + 2 >= a.t0 + 3) {
                    if (t + 2 <= t_terms && lane < kXTerms / 4) reinterpret_cast<f4v *>(RING(t + 2))[lane] = pre_terms;
                    if (t + 2 < a.L && lane < 11) NZ(t + 2)[lane] = mol_noise_term(pre_noise, lane);
                }
                if (t + 3 <= t_terms && lane < kXTerms / 4) pre_terms = reinterpret_cast<const f4v *>(TERMS(t + 3))[lane];
                if (t + 3 < a.L && lane < 11)
                    pre_noise = a.noise ? a.noise[((size_t)(t + 3) * a.Bt + b) * 11 + lane]
                                        : philox_noise(a.seed, prow, (uint32_t)(t + 3), (uint32_t)lane, 1);
            }
        }
        bar();
        if (*abort_flag) return;
        if (wave != 0) x = xs[t & 1];
    }
    // ---- carry the recurrent state to the next time chunk (every workgroup its own copy)
    __syncthreads();
    st[tid] = h1v;
    for (int i = tid; i < 4 * R; i += kXThreads) st[512 + i] = sg[i];
    if (tid < 48) st[512 + 2048 + tid] = gh2s[tid];
    if (lane < 2) st[512 + 2048 + 48 + ui] = h2own;
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
