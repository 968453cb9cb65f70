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

// diagnostics (tools/ab_libs.sh): skip an off-critical exchange (wrong results, timing only)
#ifndef WRNN_XCD_SKIP_SG
#define WRNN_XCD_SKIP_SG 0
#endif
#ifndef WRNN_XCD_SKIP_H2
#define WRNN_XCD_SKIP_H2 0
#endif
#ifndef WRNN_XCD_FAST_EXP
#define WRNN_XCD_FAST_EXP 1     // sampler scale e^s by v_exp_f32 (A/B vs libm expf: 3.92 -> 3.88 us/step, parity unchanged)
#endif
#ifndef WRNN_XCD_PRIO
#define WRNN_XCD_PRIO 0         // s_setprio of wave 0 (the poller / sampler)
#endif

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

// MoL sampler (utils/distribution.py:87-123) on logits held in pairs: lane jp (of every DPP row)
// holds logits 2jp (la) and 2jp+1 (lb); ua / ub = log(-log u1) of those mixture indices (jp < 5).
// k = argmax over the 10 logit_probs − u (first max on ties), then the logistic draw with the
// selected mean (logit 10 + k) and log-scale (logit 20 + k).  Result wave-uniform.
__device__ __forceinline__ float mol_sample_pairs(float la, float lb, float ua, float ub, float u10, int jp) {
    float v = -INFINITY;
    int i = 64;
    if (jp < 5) {
        const float va = la - ua, vb = lb - ub;
        const bool hi = vb > va;                    // tie → the smaller index
        v = hi ? vb : va;
        i = 2 * jp + (hi ? 1 : 0);
    }
#define WRNN_AM_STAGE(ctrl)                                                           \
    {                                                                                 \
        float ov = WRNN_DPP(v, ctrl);                                                 \
        int oi = __builtin_amdgcn_mov_dpp(i, (ctrl), 0xF, 0xF, false);                \
        am_merge(v, i, ov, oi);                                                       \
    }
    WRNN_AM_STAGE(0xB1) WRNN_AM_STAGE(0x4E) WRNN_AM_STAGE(0x141) WRNN_AM_STAGE(0x140)
#undef WRNN_AM_STAGE
    const int k = __builtin_amdgcn_readlane(i, 0);
    const int km = (10 + k) >> 1, ks = (20 + k) >> 1;     // lanes of logits 10 + k, 20 + k (same parity as k)
    const float ma = lane_bcast(la, km), mb = lane_bcast(lb, km), sa = lane_bcast(la, ks), sb = lane_bcast(lb, ks);
    const float mean = (k & 1) ? mb : ma;
    const float ls = fmaxf((k & 1) ? sb : sa, -32.23619130191664f);
#if WRNN_XCD_FAST_EXP
    float x = mean + fast_exp(ls) * u10;
#else
    float x = mean + expf(ls) * u10;
#endif
    x = x < -1.0f ? -1.0f : x;
    x = x > 1.0f ? 1.0f : x;
    return x;
}

// 32-lane dot engine: a wave is two engines (e = lane >> 5), each computing one 512-long row per
// pass; lane li = lane & 31 of an engine holds the float4 chunks li + 32m (m = 0..3) of its row
// (16 weights) and reads the same chunks of x.  Packed FMAs, then Σ over the engine's 32 lanes:
// row_sum16 (DPP, identical bits in its 16 lanes) + the paired DPP row (permlane16 swap).
__device__ __forceinline__ float e32dot(const f4v (&w)[4], const f4v (&x)[4]) {
    f2v a = __builtin_elementwise_fma(w[0].xy, x[0].xy, f2v{0.0f, 0.0f});
    f2v b = __builtin_elementwise_fma(w[1].xy, x[1].xy, f2v{0.0f, 0.0f});
    a = __builtin_elementwise_fma(w[0].zw, x[0].zw, a);
    b = __builtin_elementwise_fma(w[1].zw, x[1].zw, b);
    a = __builtin_elementwise_fma(w[2].xy, x[2].xy, a);
    b = __builtin_elementwise_fma(w[3].xy, x[3].xy, b);
    a = __builtin_elementwise_fma(w[2].zw, x[2].zw, a);
    b = __builtin_elementwise_fma(w[3].zw, x[3].zw, b);
    const f2v s = a + b;
    return perm_sum16(row_sum16(s.x + s.y));
}

__device__ __forceinline__ f4v lds4(const float *p) { return *reinterpret_cast<const f4v *>(p); }

// x chunks of an engine lane (li = lane & 31) from a 512-float LDS vector
__device__ __forceinline__ void e32x(const float *v, int li, f4v (&x)[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) x[m] = lds4(v + 4 * (li + 32 * m));
}

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


typedef unsigned u4v __attribute__((ext_vector_type(4)));

// A hop vector as a raw buffer: 16-byte sc1 loads (two granules each, every 8-byte half untorn:
// MI355X_MICROARCH.md hand-off table), lane offset + instruction immediate
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hop_rsrc(const unsigned long long *g) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned long long *>(g), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ u4v ld16_sc1(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16 /* sc1 */);
}

// Poll NP·128 granules (pairs l + 64k, k < NP) with 16-byte loads until every granule carries
// `tag`, then store2(i, v_i, v_i+1) for each pair's first granule index i.  Bounded.
template <int NP, typename Store2>
__device__ __forceinline__ void xgather16(const unsigned long long *g, uint32_t tag, int *ctl, long long timeout,
                                          int step, int hop, int *lds_abort, int lid, Store2 store2) {
    const __amdgpu_buffer_rsrc_t r = hop_rsrc(g);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (;;) {
        u4v v[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) v[k] = ld16_sc1(r, 16 * (lid + 64 * k));
        bool ok = true;
#pragma unroll
        for (int k = 0; k < NP; ++k) ok &= (v[k].y == tag) & (v[k].w == tag);
        if (ok) {
#pragma unroll
            for (int k = 0; k < NP; ++k) store2(2 * (lid + 64 * k), __uint_as_float(v[k].x), __uint_as_float(v[k].z));
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

#define XSTAMPW(kk, w)                                                                                        \
    do {                                                                                                      \
        if (kDbg && a.dbg && wave == (w) && lane == 0 && t - a.t0 < a.dbg_steps)                              \
            a.dbg[((size_t)mem * a.dbg_steps + (t - a.t0)) * kStamps + (kk)] = (unsigned)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define XSTAMP(kk) XSTAMPW(kk, 0)

template <bool kDbg>
__global__ __launch_bounds__(kXThreads, 2) void fatchord_xcd_kernel(XcdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int R = 512, NC = 30, TW = kXcdWgs * kXTerms;
    const XcdLds ll = xcd_lds_layout();
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 31, eng = lane >> 5;
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

    // ---- register-resident weights: engine e of wave w holds, per pass, one row's chunks li + 32m
    //   GRU2: pass q = gate q of unit 2w + e (slab row 2q + e);  fc1 / fc2: row 2w + e;
    //   W_hh2 (waves 1..7): pass p = row (w-1)·4 + 2p + e
    f4v wih2[3][4], w1r[4], w2r[4], whh2r[2][4];
    auto ldrow = [&](const float *row, int m) { return *reinterpret_cast<const f4v *>(row + 4 * (li + 32 * m)); };
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int q = 0; q < 3; ++q) wih2[q][m] = ldrow(S + a.s.wih2 + (wave * 6 + 2 * q + eng) * R, m);
        w1r[m] = ldrow(S + a.s.w1 + (wave * 2 + eng) * R, m);
        w2r[m] = ldrow(S + a.s.w2 + (wave * 2 + eng) * R, m);
#pragma unroll
        for (int p = 0; p < 2; ++p)
            whh2r[p][m] = wave >= 1 ? ldrow(S + a.s.whh2 + ((wave - 1) * kXH2Reg + 2 * p + eng) * R, m)
                                    : f4v{0.0f, 0.0f, 0.0f, 0.0f};
    }
    const float w3a = S[a.s.w3 + (wave * 2 + 0) * 32 + li];
    const float w3b = S[a.s.w3 + (wave * 2 + 1) * 32 + li];
    // GRU1 of unit tid: x-coefficients
    const float q1r = S[a.s.q1a + tid], q1z = S[a.s.q1a + R + tid], q1n = S[a.s.q1a + 2 * R + tid];
    const int ui = wave * 2 + eng;                   // this engine's local unit and fc row
    // W_hh1 rows (waves 1..5 and 7, eight each): gh0 + 2p + e, p = 0..3; lane li < 4 of an
    // engine publishes the terms of its row 2·li + e
    const bool gh1w = wave >= 1 && wave != 6;
    const int gh0 = 8 * (wave <= 5 ? wave - 1 : 5);
    const int h2l0 = (wave - 1) * 3;                 // W_hh2 LDS rows of waves 1..7: 28 + h2l0 + {0, 1, 2}

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
        unsigned long long *g = XG(XH_S0 + (t & 1)) + (size_t)(c * kXUnits + u) * 4;
        const uint32_t tag = (uint32_t)t + 1u;
        if (q < 2) {
            xpub(g + q, tag, (gh + bh) + (p1 + bi));
        } else {
            xpub(g + 3, tag, gh + bh);
            xpub(g + 2, tag, p1 + bi);
        }
    };
    // the GRU1 terms of this wave's 8 W_hh1 rows (gh[p]: row gh0 + 2p + e), lanes li < 4
    auto publish_terms = [&](int t, const float (&gh)[4]) {
        if (li < 4) {
            const float v = li == 0 ? gh[0] : li == 1 ? gh[1] : li == 2 ? gh[2] : gh[3];
            publish_term(t, gh0 + 2 * li + eng, v);
        }
    };
    // a quarter of step t's GRU1 terms (waves 3..6: 512 granules each, one poll round)
    auto gather_terms = [&](int t) {
        const int qq = wave - 3;
        xgather16<4>(XG(XH_S0 + (t & 1)) + qq * 512, (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t, XH_S0 + (t & 1),
                     abort_flag, lane, [&](int i, float v0, float v1) {
                         *reinterpret_cast<f2v *>(sg + qq * 512 + i) = f2v{v0, v1};
                     });
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
    float h2own = resume ? st[512 + 2048 + 48 + ui] : 0.0f;   // h2 of this engine's unit
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
            const float z4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            publish_terms(0, z4);
        }
        if (wave >= 3 && wave <= 6) {
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
            const float h1j = h1s[c * kXUnits + ui];
            const float g_r = e32dot(wih2[0], hx), g_z = e32dot(wih2[1], hx), g_n = e32dot(wih2[2], hx);
            const float hn = gru_gate_math(g_r + p2q[0], g_z + p2q[1], g_n + p2q[2], ghv[0], ghv[1], ghv[2], h2own);
            h2own = hn;
            // y = (x_I + h1) + h2 (:212, :216)
            const float y = (xi + h1j) + hn;
            if (li == 0) {
                xpub(XG(XH_Y) + c * kXUnits + ui, tag, y);
                xpub(XG(XH_H2) + c * kXUnits + ui, tag, hn);
            }
        }
        XSTAMP(2);
        // ---- hop Y (wave 0) ‖ W_hh1·h1 → GRU1 terms of step t+1 (waves 1..7)
        if (wave == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            xgather16<4>(XG(XH_Y), tag, a.ctl, a.timeout_ticks, t, XH_Y, abort_flag, lane,
                         [&](int i, float v0, float v1) { *reinterpret_cast<f2v *>(ys + i) = f2v{v0, v1}; });
            XSTAMP(3);
        } else if (wave == 6) {
            if (more && !WRNN_XCD_SKIP_H2) {   // h2 (published with y) for the W_hh2 dots of the next window
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                xgather16<4>(XG(XH_H2), tag, a.ctl, a.timeout_ticks, t, XH_H2, abort_flag, lane,
                             [&](int i, float v0, float v1) { *reinterpret_cast<f2v *>(h2s + i) = f2v{v0, v1}; });
            }
            XSTAMPW(10, 6);
        } else if (more) {
            // W_hh1·h1 → GRU1 terms of step t+1: the 4 dots first (LDS reads of later rows overlap
            // earlier dots), then one publish
            f4v hx[4];
            e32x(h1s, li, hx);
            float gh[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                f4v wr[4];
                e32x(whh1 + (gh0 + 2 * p + eng) * R, li, wr);
                gh[p] = e32dot(wr, hx);
            }
            publish_terms(t + 1, gh);
            XSTAMPW(9, 1);
        }
        const float v1 = tr[XT_V1 + ui], v2 = tr[XT_V2 + ui];
        bar();
        XSTAMPW(14, 3);
        // ---- fc1 (:216-218), row ui → relu → hop F1
        {
            f4v yx[4];
            e32x(ys, li, yx);
            const float A = e32dot(w1r, yx) + v1;
            if (li == 0) xpub(XG(XH_F1) + c * kXFcRows + ui, tag, A > 0.0f ? A : 0.0f);
        }
        XSTAMP(4);
        if (wave == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            xgather16<4>(XG(XH_F1), tag, a.ctl, a.timeout_ticks, t, XH_F1, abort_flag, lane,
                         [&](int i, float v0, float v1) { *reinterpret_cast<f2v *>(f1s + i) = f2v{v0, v1}; });
            XSTAMP(5);
        } else if (more) {
            // W_hh2·h2 → gh2s for the next GRU2: passes 0/1 the VGPR rows, 2/3 the LDS rows
            // 28 + h2l0 + {0, 1, 2}; all dots first, then the LDS stores
            f4v hx[4];
            e32x(h2s, li, hx);
            float gh[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                if (p < 2) {
                    gh[p] = e32dot(whh2r[p], hx);
                } else {
                    const int lr = h2l0 + 2 * (p - 2) + eng;     // wave 7 has LDS rows 18, 19 only
                    f4v wr[4];
                    e32x(whh2l + (lr < 48 - kXH2RegRows ? lr : 48 - kXH2RegRows - 1) * R, li, wr);
                    gh[p] = e32dot(wr, hx);
                }
            }
            if (li < 4) {
                const int lr = h2l0 + 2 * (li - 2) + eng;
                const int rr = li < 2 ? (wave - 1) * kXH2Reg + 2 * li + eng
                                      : ((2 * (li - 2) + eng < 3 && lr < 48 - kXH2RegRows) ? kXH2RegRows + lr : -1);
                const float v = li == 0 ? gh[0] : li == 1 ? gh[1] : li == 2 ? gh[2] : gh[3];
                if (rr >= 0) gh2s[rr] = v;
            }
            XSTAMPW(13, 3);
        }
        bar();
        // ---- fc2 (:220-221) → relu → fc3 partial logits of the 16 own f2 rows (:223)
        {
            f4v fx[4];
            e32x(f1s, li, fx);
            float A = e32dot(w2r, fx) + v2;
            A = A > 0.0f ? A : 0.0f;
            const float f20 = lane_bcast(A, 0), f21 = lane_bcast(A, 32);
            if (lane < 32) part[wave * 32 + lane] = fmaf(w3b, f21, w3a * f20);
        }
        bar();
        XSTAMP(6);
        if (wave == 0) {
            // Σ of the 8 waves' partials → hop F2 → Σ of the 32 workgroups' partials + b3 → sample
            if (lane < kXF2Line) {   // all 32 granules of the line (30, 31: zero weights) for the 16-byte polls
                float s = 0.0f;
#pragma unroll
                for (int w = 0; w < kXWaves; ++w) s += part[w * 32 + lane];
                xpub(XG(XH_F2) + c * kXF2Line + lane, tag, s);
            }
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
            float pa[8], pb[8];
            for (;;) {
                // the polled pieces live in whh2r's registers: wave 0 holds no W_hh2 rows (one
                // register set serves both roles, so the kernel fits 256 VGPRs)
                u4v *v = reinterpret_cast<u4v *>(&whh2r[0][0]);
#pragma unroll
                for (int m = 0; m < 8; ++m) v[m] = ld16_sc1(rf, goff + m * kXF2Line * 8);
                bool ok = true;
#pragma unroll
                for (int m = 0; m < 8; ++m) ok &= (v[m].y == tag) & (v[m].w == tag);
                if (ok) {
#pragma unroll
                    for (int m = 0; m < 8; ++m) {
                        pa[m] = __uint_as_float(v[m].x);
                        pb[m] = __uint_as_float(v[m].z);
                    }
                    break;
                }
                if ((++spins & 63u) == 0) {
                    const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                    const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    if (late || other) {
                        if (late) record_abort(a.ctl, -4, t, XH_F2, blockIdx.x);
                        *abort_flag = 1;
#pragma unroll
                        for (int m = 0; m < 8; ++m) pa[m] = pb[m] = 0.0f;
                        break;
                    }
                }
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
            const float la = cross_rows(pa[0]) + b3a, lb = cross_rows(pb[0]) + b3b;   // logits 2jp, 2jp+1
            x = mol_sample_pairs(la, lb, ua, ub, u10, jp);
            if (lane == 0) {
                xs[t & 1] = x;
                if (c == 0) a.out[(size_t)b * a.L + t] = x;
            }
            XSTAMP(8);
        } else if (more) {
            if (wave >= 3 && wave <= 6 && !WRNN_XCD_SKIP_SG) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                gather_terms(t + 1);
                XSTAMPW(11, 5);
            }
            if (wave == 7 && t + 2 >= a.t0 + 3) {
                // ring: step t+2's terms and sampler noise, loaded and stored within this window
                // (the longest of the step; a load carried across steps in registers would not
                // fit the VGPR budget, and an LDS-DMA makes hipcc wait for it before every later
                // LDS access of the issuing wave)
                if (t + 2 <= t_terms && lane < kXTerms / 4)
                    reinterpret_cast<f4v *>(RING(t + 2))[lane] = reinterpret_cast<const f4v *>(TERMS(t + 2))[lane];
                if (t + 2 < a.L && lane < 11) NZ(t + 2)[lane] = noise_term(t + 2);
                XSTAMPW(12, 7);
            }
        }
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
