// xcd_device.h — device helpers of the XCD-resident kernels (fatchord_xcd.hip, dense rnn 512;
// fatchord_xcds.hip, block-sparse rnn 896): XCD membership, XCD-local granule publishes, 16-byte
// sc1 polls, cross-row sums, the in-register fc rows of a polled vector, the MoL sampler.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wrnn_device.h"

namespace wrnn {

#ifndef WRNN_XCD_ORDERED_ARGMAX
#define WRNN_XCD_ORDERED_ARGMAX 1   // MoL argmax: value-only max over lanes 0..7 + ballot (0: index through DPP)
#endif
#ifndef WRNN_XCD_UNIFORM_WAVE
#define WRNN_XCD_UNIFORM_WAVE 1   // the XCD kernels' wave index through readfirstlane (0: per-lane, A/B)
#endif
#ifndef WRNN_XCD_BAR_STAMPS
#define WRNN_XCD_BAR_STAMPS 0     // stamped diagnostic builds: each wave's arrival at the step-end barrier
#endif
#ifndef WRNN_XCD_LEAN_SAMPLER
#define WRNN_XCD_LEAN_SAMPLER 1   // sampler: both logit sums through one permlane chain, med3 clamps, max + DPP as one instruction
#endif
#ifndef WRNN_XCD_FAST_EXP
#define WRNN_XCD_FAST_EXP 1     // sampler scale e^s by v_exp_f32 (A/B vs libm expf: 3.92 -> 3.88 us/step, parity unchanged)
#endif

__device__ __forceinline__ unsigned xcc_id() {
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xF;   // HW_REG_XCC_ID[3:0]
}

// XCD-local publish: a plain (workgroup-scope) 8-byte store keeps the line in this XCD's L2
__device__ __forceinline__ void xpub(unsigned long long *g, uint32_t tag, float v) {
    const unsigned long long x = ((unsigned long long)tag << 32) | __float_as_uint(v);
    __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The same publish through a buffer resource over the XCD's hop area (one wave-uniform
// descriptor; the per-lane part is a 32-bit granule index instead of a 64-bit address — fewer
// VGPRs live across the step loop).  Plain buffer store: no cache bits, as xpub.
typedef unsigned u2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void xpub_b(__amdgpu_buffer_rsrc_t r, int granule, uint32_t tag, float v) {
    __builtin_amdgcn_raw_buffer_store_b64(u2v{__float_as_uint(v), tag}, r, granule * 8, 0, 0);
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
// cross_rows of two values at once (the same sums, bit for bit: (r0 + r1) + (r2 + r3)): the
// permlane16 swap of (a, b) leaves the row-pair sums of a in one row of each pair and those of b
// in the other, permlane32 adds the pairs, a last permlane16 swap spreads each total to every row
// (whichever way the swap pairs its rows, a ends in its first result).  3 permlanes + 2 adds
// instead of 4 + 4.
__device__ __forceinline__ void cross_rows2(float &a, float &b) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    const float p = __uint_as_float(s[0]) + __uint_as_float(s[1]);
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(p), __float_as_uint(p), false, false);
    const float r = __uint_as_float(q[0]) + __uint_as_float(q[1]);
    const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(r), __float_as_uint(r), false, false);
    a = __uint_as_float(t[0]);
    b = __uint_as_float(t[1]);
}
__device__ __forceinline__ void cross_rows_pair(float &a, float &b) {
    if (WRNN_XCD_LEAN_SAMPLER) {
        cross_rows2(a, b);
    } else {
        a = cross_rows(a);
        b = cross_rows(b);
    }
}
// max over each 8-lane group (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror), one v_max_f32
// with the DPP source per stage (hipcc emits mov_dpp + a canonicalising max + max); the s_nop 1
// covers the VALU-write → DPP-read hazard the compiler does not see inside the asm
__device__ __forceinline__ float max8_dpp(float v) {
    float r;
    asm volatile(
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=&v"(r)
        : "v"(v));
    return r;
}

// MoL sampler (utils/distribution.py:87-123) on logits held in pairs: lane jp (of every DPP row)
// holds logits 2jp (la) and 2jp+1 (lb); ua / ub = log(-log u1) of those mixture indices (jp < 5).
// k = argmax over the 10 logit_probs − u (first max on ties), then the logistic draw with the
// selected mean (logit 10 + k) and log-scale (logit 20 + k).  The draws of all ten components are
// formed beside the argmax (lanes 5..9 hold the means of k = 2(jp − 5) + {0, 1}, row_shl:5 brings
// the matching log-scales from lanes 10..14), so only a lane read follows it.  Result wave-uniform.
__device__ __forceinline__ float mol_sample_pairs(float la, float lb, float ua, float ub, float u10, int jp) {
    // row_shl:5: lane jp + 5; max with the clamp bound (med3 with +inf: the same for every
    // non-NaN value, without fmaxf's canonicalising extra max)
    const float sa = WRNN_XCD_LEAN_SAMPLER ? __builtin_amdgcn_fmed3f(WRNN_DPP(la, 0x105), -32.23619130191664f, INFINITY)
                                           : fmaxf(WRNN_DPP(la, 0x105), -32.23619130191664f);
    const float sb = WRNN_XCD_LEAN_SAMPLER ? __builtin_amdgcn_fmed3f(WRNN_DPP(lb, 0x105), -32.23619130191664f, INFINITY)
                                           : fmaxf(WRNN_DPP(lb, 0x105), -32.23619130191664f);
#if WRNN_XCD_FAST_EXP
    float xa = la + fast_exp(sa) * u10, xb = lb + fast_exp(sb) * u10;
#else
    float xa = la + expf(sa) * u10, xb = lb + expf(sb) * u10;
#endif
    if (WRNN_XCD_LEAN_SAMPLER) {   // (finite x: the same clamp)
        xa = __builtin_amdgcn_fmed3f(xa, -1.0f, 1.0f);
        xb = __builtin_amdgcn_fmed3f(xb, -1.0f, 1.0f);
    } else {
        xa = xa < -1.0f ? -1.0f : xa;
        xa = xa > 1.0f ? 1.0f : xa;
        xb = xb < -1.0f ? -1.0f : xb;
        xb = xb > 1.0f ? 1.0f : xb;
    }
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
    int k;
    if constexpr (WRNN_XCD_ORDERED_ARGMAX) {
        // the components grow with the lane (lane jp: 2jp, 2jp + 1), so the winner is the first of
        // lanes 0..4 holding the max: three value-only DPP stages cover lanes 0..7 (every DPP row
        // holds the same bits), a ballot finds the lane (wave_argmax_ordered, specialised)
        float mv;
        if (WRNN_XCD_LEAN_SAMPLER) {
            mv = max8_dpp(v);
        } else {
            mv = fmaxf(v, WRNN_DPP(v, 0xB1));
            mv = fmaxf(mv, WRNN_DPP(mv, 0x4E));
            mv = fmaxf(mv, WRNN_DPP(mv, 0x141));
        }
        const float m = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, mv)));
        const unsigned long long hit = __ballot(v == m) & 0x1Full;
        if (hit != 0) {
            k = __builtin_amdgcn_readlane(i, (int)__builtin_ctzll(hit));
        } else {   // every logit NaN (fmaxf skips NaN operands, so a single NaN never wins): fallback
            WRNN_AM_STAGE(0xB1) WRNN_AM_STAGE(0x4E) WRNN_AM_STAGE(0x141) WRNN_AM_STAGE(0x140)
            k = __builtin_amdgcn_readlane(i, 0);
        }
    } else {
        WRNN_AM_STAGE(0xB1) WRNN_AM_STAGE(0x4E) WRNN_AM_STAGE(0x141) WRNN_AM_STAGE(0x140)
        k = __builtin_amdgcn_readlane(i, 0);
    }
#undef WRNN_AM_STAGE
    return lane_bcast((k & 1) ? xb : xa, 5 + (k >> 1));
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

// The in-lane part of e32dot (no cross-lane sum)
__device__ __forceinline__ float e32part(const f4v (&w)[4], const f4v (&x)[4]) {
    f2v a = __builtin_elementwise_fma(w[0].xy, x[0].xy, f2v{0.0f, 0.0f});
    f2v b = __builtin_elementwise_fma(w[1].xy, x[1].xy, f2v{0.0f, 0.0f});
    a = __builtin_elementwise_fma(w[0].zw, x[0].zw, a);
    b = __builtin_elementwise_fma(w[1].zw, x[1].zw, b);
    a = __builtin_elementwise_fma(w[2].xy, x[2].xy, a);
    b = __builtin_elementwise_fma(w[3].xy, x[3].xy, b);
    a = __builtin_elementwise_fma(w[2].zw, x[2].zw, a);
    b = __builtin_elementwise_fma(w[3].zw, x[3].zw, b);
    const f2v s = a + b;
    return s.x + s.y;
}

// Three e32dot rows of an engine (the r, z, n gate rows of its unit) reduce-scattered over its 32
// lanes: lane l keeps row l & 3 (a zero fourth row) against l ^ 1, then l ^ 2, then sums the
// lanes of its residue class (row_ror 4 and 8, the paired DPP row); lanes 1 and 2 hand z and n
// to lane 0.  8 cross-lane operations on one chain instead of 3 × 5.  Valid in lanes li == 0.
__device__ __forceinline__ void e32dot3_rs(const f4v (&w0)[4], const f4v (&w1)[4], const f4v (&w2)[4],
                                           const f4v (&x)[4], int lane, float &gr, float &gz, float &gn) {
    const float t0 = e32part(w0, x), t1 = e32part(w1, x), t2 = e32part(w2, x);
    const bool odd = (lane & 1) != 0, hi = (lane & 2) != 0;
    const float u0 = odd ? t1 : t0, v0 = odd ? t0 : t1;
    const float u1 = odd ? 0.0f : t2, v1 = odd ? t2 : 0.0f;
    const float a0 = u0 + WRNN_DPP(v0, 0xB1), a1 = u1 + WRNN_DPP(v1, 0xB1);   // quad_perm [1,0,3,2]
    const float keep = hi ? a1 : a0, send = hi ? a0 : a1;
    float b = keep + WRNN_DPP(send, 0x4E);                                     // quad_perm [2,3,0,1]
    b += WRNN_DPP(b, 0x124);                                                   // row_ror:4
    b += WRNN_DPP(b, 0x128);                                                   // row_ror:8
    b = perm_sum16(b);
    gr = b;
    gz = WRNN_DPP(b, 0x55);   // quad_perm [1,1,1,1]
    gn = WRNN_DPP(b, 0xAA);   // quad_perm [2,2,2,2]
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
        if (__ballot(!ok) == 0) {   // wave-uniform exit (a per-lane exit builds exec-mask branches)
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
        if (__ballot(!ok) == 0) {
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

// Poll NP·128 granules (pairs l + 64k) with 16-byte loads until every granule carries `tag`;
// the pairs stay in registers (v[k].x, v[k].z).  Bounded; on abort the values are garbage.
template <int NP>
__device__ __forceinline__ void xpoll16(const unsigned long long *g, uint32_t tag, int *ctl, long long timeout,
                                        int step, int hop, int *lds_abort, int lid, u4v (&v)[NP]) {
    const __amdgpu_buffer_rsrc_t r = hop_rsrc(g);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (;;) {
#pragma unroll
        for (int k = 0; k < NP; ++k) v[k] = ld16_sc1(r, 16 * (lid + 64 * k));
        bool ok = true;
#pragma unroll
        for (int k = 0; k < NP; ++k) ok &= (v[k].y == tag) & (v[k].w == tag);
        if (__ballot(!ok) == 0) return;
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

// 8 rows of a 512-wide layer against a vector polled into registers by ONE wave (no LDS, no
// barrier): lane l holds the pairs k = 0..3 at granules 2(l + 64k) + {0, 1} (xk[k]) and the
// matching weights of row r in w[2r + k/2] (.xy for even k, .zw for odd).  Packed FMAs, then a
// reduce-scatter over the wave — permlane32 swap (row r vs r + 4), permlane16 swap (r vs r + 2),
// DPP sum over the 16 lanes of a row — leaves in o[j] the full sum of row j + 2·(l >> 4),
// identical bits in all 16 lanes of DPP row l >> 4.
__device__ __forceinline__ void fc8_rows(const f4v (&w)[16], const f2v (&xk)[4], float (&o)[2]) {
    float s[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        f2v acc = __builtin_elementwise_fma(w[2 * r].xy, xk[0], f2v{0.0f, 0.0f});
        f2v acc2 = __builtin_elementwise_fma(w[2 * r].zw, xk[1], f2v{0.0f, 0.0f});
        acc = __builtin_elementwise_fma(w[2 * r + 1].xy, xk[2], acc);
        acc2 = __builtin_elementwise_fma(w[2 * r + 1].zw, xk[3], acc2);
        const f2v t = acc + acc2;
        s[r] = t.x + t.y;
    }
    float h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // lanes < 32 keep row j, lanes ≥ 32 row j + 4
        const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s[j]), __float_as_uint(s[j + 4]), false, false);
        h[j] = __uint_as_float(q[0]) + __uint_as_float(q[1]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {   // even DPP rows keep h[j], odd rows h[j + 2]
        const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(h[j]), __float_as_uint(h[j + 2]), false, false);
        o[j] = row_sum16(__uint_as_float(q[0]) + __uint_as_float(q[1]));
    }
}

}  // namespace wrnn
