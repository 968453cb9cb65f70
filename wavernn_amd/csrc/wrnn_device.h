// wrnn_device.h — device helpers shared by the WaveRNN loop kernels (fatchord_loop.hip,
// fatchord_rows.hip): DPP wave/row reductions, gate nonlinearities, Philox, hand-off
// granules and bounded polls, the LDS-only barrier.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wrnn {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ wave-level helpers
// (update_dpp with old = 0 and bound_ctrl: hipcc then folds the move into the consuming VALU op,
// v_add_f32_dpp instead of v_mov_b32_dpp + v_add_f32).  quad_perm, the row mirrors and row_ror
// always read a valid lane; the row shifts (row_shl / row_shr, e.g. xcd_device.h's row_shl:5)
// do not: their out-of-row lanes read 0 here, not their old value — callers must not select
// those lanes)
#define WRNN_DPP(v, ctrl) \
    __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, (v)), (ctrl), 0xF, 0xF, true))

// Full-wave sum; every lane returns the same bits.  Row stages via DPP (xor1, xor2,
// half-mirror, mirror), then the four row sums combined in a fixed order.
__device__ __forceinline__ float wave_sum(float v) {
    v += WRNN_DPP(v, 0xB1);    // quad_perm [1,0,3,2]
    v += WRNN_DPP(v, 0x4E);    // quad_perm [2,3,0,1]
    v += WRNN_DPP(v, 0x141);   // row_half_mirror
    v += WRNN_DPP(v, 0x140);   // row_mirror
    float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
    float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
    float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
    return (r0 + r1) + (r2 + r3);
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, WRNN_DPP(v, 0xB1));
    v = fmaxf(v, WRNN_DPP(v, 0x4E));
    v = fmaxf(v, WRNN_DPP(v, 0x141));
    v = fmaxf(v, WRNN_DPP(v, 0x140));
    float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
    float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
    float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// (value, index) argmax: larger value wins, ties go to the smaller index (torch: first max).
__device__ __forceinline__ void am_merge(float &v, int &i, float ov, int oi) {
    // branch-free (bitwise, not short-circuit): hipcc otherwise emits exec-mask branches per stage
    const bool take = (ov > v) | ((ov == v) & (oi < i));
    v = take ? ov : v;
    i = take ? oi : i;
}

__device__ __forceinline__ int wave_argmax(float v, int i) {
#define WRNN_AM_STAGE(ctrl)                                                           \
    {                                                                                 \
        float ov = WRNN_DPP(v, ctrl);                                                 \
        int oi = __builtin_amdgcn_mov_dpp(i, (ctrl), 0xF, 0xF, false);                \
        am_merge(v, i, ov, oi);                                                       \
    }
    WRNN_AM_STAGE(0xB1) WRNN_AM_STAGE(0x4E) WRNN_AM_STAGE(0x141) WRNN_AM_STAGE(0x140)
#undef WRNN_AM_STAGE
    float bv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        float ov = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), r));
        int oi = __builtin_amdgcn_readlane(i, r);
        am_merge(bv, bi, ov, oi);
    }
    return bi;
}

// wave_argmax for layouts whose indices grow with the lane (every index of lane l below every
// index of lane l + 1, each lane's own candidates merged by am_merge in index order): the same
// winner — largest value, ties to the smallest index — from a value-only max reduction and the
// first lane holding it (ballot), instead of carrying the index through every DPP stage.
// NaN: fmaxf drops NaN operands, so a NaN candidate never wins here — the winner is the argmax
// over the non-NaN values (torch.argmax would return the NaN's index; the general (value, index)
// reduction below is not NaN-faithful either).  NaN logits only come from NaN weights or inputs,
// which are outside the parity contract.  The fallback runs only if every value is NaN.
__device__ __forceinline__ int wave_argmax_ordered(float v, int i) {
    const float m = wave_max(v);
    const unsigned long long hit = __ballot(v == m);
    if (hit == 0) return wave_argmax(v, i);
    return __builtin_amdgcn_readlane(i, (int)__builtin_ctzll(hit));
}

// wave_argmax for any layout: a value-only max reduction, then the lane holding it (ballot); only
// when several lanes hold the maximum (an exact tie across lanes) does the (value, index)
// reduction decide.  Same winner as wave_argmax for finite values (NaN: as wave_argmax_ordered,
// a NaN candidate is skipped unless every value is NaN).
__device__ __forceinline__ int wave_argmax_fast(float v, int i) {
    const float m = wave_max(v);
    const unsigned long long hit = __ballot(v == m);
    if (__builtin_popcountll(hit) == 1) return __builtin_amdgcn_readlane(i, (int)__builtin_ctzll(hit));
    return wave_argmax(v, i);
}

// NR dot products against one shared vector: acc[r] += W[r]·x over K4 float4 chunks,
// row r at w0 + r·wstride.  Lane l takes chunks l, l+64, … (contiguous 16 B per lane:
// conflict-free ds_read_b128).
template <int NR>
__device__ __forceinline__ void dots(const float *__restrict__ w0, int wstride, const float *__restrict__ x,
                                     int K4, int lane, float (&acc)[NR]) {
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
#pragma unroll 4
    for (int c = lane; c < K4; c += 64) {
        const float4 xv = x4[c];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const float4 wv = reinterpret_cast<const float4 *>(w0 + r * wstride)[c];
            float a = acc[r];
            a = fmaf(wv.x, xv.x, a);
            a = fmaf(wv.y, xv.y, a);
            a = fmaf(wv.z, xv.z, a);
            a = fmaf(wv.w, xv.w, a);
            acc[r] = a;
        }
    }
}

// Gate nonlinearities on the critical path use the hardware exp2 (v_exp_f32) and reciprocal:
// ≈1e-7 absolute error, inside the parity tolerance (the reference's SLEEF/MKL paths are not
// correctly rounded either).  Samplers keep the accurate libm functions.
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
// The deepmind input x = c / 127.5 − 1 of a label c ∈ {0, …, 255} (deepmind_version.py:106-108,
// :135-136) with the IEEE quotient: one FMA correction of c·fl(1/127.5) rounds correctly for every
// label (checked exhaustively, tests/test_label_x.py), 4 instructions instead of the division
// sequence (v_div_scale / rcp / 5 FMAs / div_fmas / div_fixup) on the gates' critical path.
__device__ __forceinline__ float label_x(float c) {
    constexpr float r = 1.0f / 127.5f;
    const float q0 = c * r;
    const float e = __builtin_fmaf(-q0, 127.5f, c);   // exact residual
    return __builtin_fmaf(e, r, q0) - 1.0f;
}
__device__ __forceinline__ float sigmoid_(float x) { return __builtin_amdgcn_rcpf(1.0f + fast_exp(-x)); }
__device__ __forceinline__ float tanh_(float x) {
    const float e = fast_exp(-2.0f * fabsf(x));            // in (0, 1]: no overflow
    const float t = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
    return copysignf(t, x);
}

// ------------------------------------------------------------------------------ Philox
__device__ __forceinline__ uint32_t philox_word(unsigned long long seed, unsigned long long row,
                                                uint32_t step, uint32_t k) {
    uint32_t c0 = k >> 2, c1 = step, c2 = (uint32_t)row, c3 = (uint32_t)(row >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    const uint32_t w = k & 3;
    return w == 0 ? c0 : w == 1 ? c1 : w == 2 ? c2 : c3;
}

// Draw k of row/step in the reference distribution (MOL: U(1e-5, 1-1e-5); RAW / DM: Exp(1)), from
// the top 24 bits of the word.  Both maps are exactly restatable on the host (oracle/philox.py):
// the MoL map is one explicit FMA (what hipcc's contraction formed from `1e-5f + c·u` anyway); the
// Exp(1) map takes the log in float64 and rounds once — the fp32 logf (v_log_f32 + scaling) read
// about one ulp high on a third of the draws (profiles/r06_philox_logf.log).  Only the fill kernel
// and the fallback kernels evaluate it; the XCD-resident kernels load filled draws.
__device__ __forceinline__ float philox_noise(unsigned long long seed, unsigned long long row,
                                              uint32_t step, uint32_t k, int mol) {
    const uint32_t w = philox_word(seed, row, step, k);
    if (mol) return __builtin_fmaf(1.0f - 2e-5f, (float)(w >> 8) * 0x1p-24f, 1e-5f);
    return (float)(-::log((double)((w >> 8) + 1u) * 0x1p-24));
}

// ---------------------------------------------------------------------------- hand-off
__device__ __forceinline__ void publish(unsigned long long *g, uint32_t tag, float v) {
    const unsigned long long x = ((unsigned long long)tag << 32) | __float_as_uint(v);
    __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __noinline__ void record_abort(int *ctl, int code, int step, int hop, int wg) {
    if (atomicCAS(&ctl[1], 0, code) == 0) {
        ctl[2] = step;
        ctl[3] = hop;
        ctl[4] = wg;
    }
    __hip_atomic_store(&ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Gather granules [base, base + NG·NL) ∩ [0, n) of one hand-off vector (n = rows·N values);
// store(b, j, v) puts each value where it belongs.  Called by NL lanes (lane id `lid`).  A
// pass issues NG UNCONDITIONAL loads (slots >= n re-read padding: the granule buffer has
// kOverRead spare granules after every vector) and only then inspects them: guarding each load
// with a runtime condition makes hipcc branch around it and wait vmcnt(0) per load, i.e. NG
// serialized memory round trips per pass (measured: 2-4x slower hops).
// On timeout, or when another workgroup has aborted, sets *lds_abort.
// kSleep > 0 backs off 64·kSleep cycles between unsuccessful polls: for off-critical vectors,
// whose polling traffic would otherwise compete with a critical hand-off in flight.
template <int NG, int NL, typename Store, int kSleep = 0>
__device__ __forceinline__ void gather(const unsigned long long *g, int base, int n, int N, uint32_t tag, int *ctl,
                                       long long timeout, int step, int hop, int *lds_abort, int lid, Store store,
                                       unsigned *dbg_slot = nullptr) {
    const unsigned long long *gp = g + base + lid;
    const int i0 = base + lid;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (;;) {
        unsigned long long v[NG];
#pragma unroll
        for (int k = 0; k < NG; ++k) v[k] = __hip_atomic_load(gp + k * NL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int k = 0; k < NG; ++k) ok &= (i0 + k * NL >= n) | ((uint32_t)(v[k] >> 32) == tag);
        if (dbg_slot && spins == 0 && lid == 0) dbg_slot[1] = (unsigned)(__builtin_amdgcn_s_memrealtime() - t0);
        if (ok) {
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const int i = i0 + k * NL;
                if (i < n) {
                    const int b = i / N;
                    store(b, i - b * N, __uint_as_float((uint32_t)v[k]));
                }
            }
            break;
        }
        if (kSleep) __builtin_amdgcn_s_sleep(kSleep);
        if ((++spins & 63u) == 0) {
            const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout;
            const bool other = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (late || other) {
                if (late) record_abort(ctl, -4, step, hop, blockIdx.x);
                *lds_abort = 1;
                break;
            }
        }
    }
    if (dbg_slot && lid == 0) dbg_slot[0] = spins + 1;
}

// gather() over a strided layout: value i sits at granule map(i) (e.g. one 128-B line per
// producer workgroup, so that no two producers' sc1 stores share a line)
template <int NG, int NL, typename Map, typename Store>
__device__ __forceinline__ void gather_mapped(const unsigned long long *g, int n, uint32_t tag, int *ctl, long long timeout,
                                              int step, int hop, int *lds_abort, int lid, Map map, Store store) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (;;) {
        unsigned long long v[NG];
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int i = lid + k * NL;
            v[k] = __hip_atomic_load(g + map(i < n ? i : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool ok = true;
#pragma unroll
        for (int k = 0; k < NG; ++k) ok &= (lid + k * NL >= n) | ((uint32_t)(v[k] >> 32) == tag);
        if (ok) {
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const int i = lid + k * NL;
                if (i < n) store(i, __uint_as_float((uint32_t)v[k]));
            }
            break;
        }
        if ((++spins & 63u) == 0) {
            const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout;
            const bool other = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (late || other) {
                if (late) record_abort(ctl, -4, step, hop, blockIdx.x);
                *lds_abort = 1;
                break;
            }
        }
    }
}

// A long, off-critical-path vector gathered in chunks of NG·NL granules (bounded registers).
template <int NG, int NL, typename Store, int kSleep = 0>
__device__ __forceinline__ void gather_chunked(const unsigned long long *g, int n, int N, uint32_t tag, int *ctl,
                                               long long timeout, int step, int hop, int *lds_abort, int lid,
                                               Store store) {
    for (int c0 = 0; c0 < n; c0 += NG * NL) {
        gather<NG, NL, Store, kSleep>(g, c0, n, N, tag, ctl, timeout, step, hop, lds_abort, lid, store);
        if (*reinterpret_cast<volatile int *>(lds_abort)) return;
    }
}

// ---- 16-lane row dots: a wave holds four DPP rows; row r (= lane >> 4) computes one dot,
// lane li (= lane & 15) of the row takes float4 chunks li, li+16, …
__device__ __forceinline__ float row_sum16(float v) {
    v += WRNN_DPP(v, 0xB1);    // quad_perm [1,0,3,2]
    v += WRNN_DPP(v, 0x4E);    // quad_perm [2,3,0,1]
    v += WRNN_DPP(v, 0x141);   // row_half_mirror
    v += WRNN_DPP(v, 0x140);   // row_mirror
    return v;                  // the row's sum, identical bits in all 16 lanes
}

__device__ __forceinline__ float row_dot(const float *__restrict__ w, const float *__restrict__ x, int K4, int li) {
    const float4 *w4 = reinterpret_cast<const float4 *>(w);
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    float acc = 0.0f;
#pragma unroll 8
    for (int c = li; c < K4; c += 16) {
        const float4 a = w4[c], b = x4[c];
        acc = fmaf(a.x, b.x, acc);
        acc = fmaf(a.y, b.y, acc);
        acc = fmaf(a.z, b.z, acc);
        acc = fmaf(a.w, b.w, acc);
    }
    return row_sum16(acc);
}

// row_dot on the critical path: packed fp32 FMAs (v_pk_fma_f32 on the aligned float4 halves)
// into four independent accumulators (even/odd chunk × xy/zw), so the per-lane chain is K4/32
// dependent packed FMAs instead of K4/4 dependent scalar ones.  Compile-time K4.
template <int K4>
__device__ __forceinline__ float row_dot_pk(const float *__restrict__ w, const float *__restrict__ x, int li) {
    static_assert(K4 % 32 == 0, "row_dot_pk: two chunks per lane per pass");
    const f4v *w4 = reinterpret_cast<const f4v *>(w) + li;
    const f4v *x4 = reinterpret_cast<const f4v *>(x) + li;
    f2v a0 = {0.0f, 0.0f}, a1 = {0.0f, 0.0f}, a2 = {0.0f, 0.0f}, a3 = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < K4 / 16; k += 2) {
        const f4v wa = w4[16 * k], xa = x4[16 * k], wb = w4[16 * (k + 1)], xb = x4[16 * (k + 1)];
        a0 = __builtin_elementwise_fma(wa.xy, xa.xy, a0);
        a1 = __builtin_elementwise_fma(wa.zw, xa.zw, a1);
        a2 = __builtin_elementwise_fma(wb.xy, xb.xy, a2);
        a3 = __builtin_elementwise_fma(wb.zw, xb.zw, a3);
    }
    const f2v s = (a0 + a1) + (a2 + a3);
    return row_sum16(s.x + s.y);
}

// Two rows against one x in a single pass (ILP for the 30-row MoL head).
__device__ __forceinline__ float2 row_dot2(const float *__restrict__ w0, const float *__restrict__ w1,
                                          const float *__restrict__ x, int K4, int li) {
    const float4 *a4 = reinterpret_cast<const float4 *>(w0);
    const float4 *b4 = reinterpret_cast<const float4 *>(w1);
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    float s0 = 0.0f, s1 = 0.0f;
#pragma unroll 8
    for (int c = li; c < K4; c += 16) {
        const float4 a = a4[c], b = b4[c], v = x4[c];
        s0 = fmaf(a.x, v.x, s0); s0 = fmaf(a.y, v.y, s0); s0 = fmaf(a.z, v.z, s0); s0 = fmaf(a.w, v.w, s0);
        s1 = fmaf(b.x, v.x, s1); s1 = fmaf(b.y, v.y, s1); s1 = fmaf(b.z, v.z, s1); s1 = fmaf(b.w, v.w, s1);
    }
    return make_float2(row_sum16(s0), row_sum16(s1));
}

__device__ __forceinline__ float lane_bcast(float v, int src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

// Whole-wave dot (one dot, 64 lanes): lane l takes chunks l, l+64, …
__device__ __forceinline__ float wave_dot(const float *__restrict__ w, const float *__restrict__ x, int K4, int lane) {
    float acc[1] = {0.f};
    dots<1>(w, 0, x, K4, lane, acc);
    return wave_sum(acc[0]);
}

// Three rows against one x in a single pass (the r/z/n gate rows of one unit).
__device__ __forceinline__ float3 row_dot3(const float *__restrict__ w0, const float *__restrict__ w1,
                                          const float *__restrict__ w2, const float *__restrict__ x, int K4, int li) {
    const float4 *a4 = reinterpret_cast<const float4 *>(w0);
    const float4 *b4 = reinterpret_cast<const float4 *>(w1);
    const float4 *c4 = reinterpret_cast<const float4 *>(w2);
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
#pragma unroll 4
    for (int c = li; c < K4; c += 16) {
        const float4 a = a4[c], b = b4[c], e = c4[c], v = x4[c];
        s0 = fmaf(a.x, v.x, s0); s0 = fmaf(a.y, v.y, s0); s0 = fmaf(a.z, v.z, s0); s0 = fmaf(a.w, v.w, s0);
        s1 = fmaf(b.x, v.x, s1); s1 = fmaf(b.y, v.y, s1); s1 = fmaf(b.z, v.z, s1); s1 = fmaf(b.w, v.w, s1);
        s2 = fmaf(e.x, v.x, s2); s2 = fmaf(e.y, v.y, s2); s2 = fmaf(e.z, v.z, s2); s2 = fmaf(e.w, v.w, s2);
    }
    return make_float3(row_sum16(s0), row_sum16(s1), row_sum16(s2));
}

// Reduce-scatter of 4 values over a 16-lane DPP row: lane l returns Σ_row p[l & 3].
// Two in-quad exchange stages (each lane keeps half of what it holds, adds its partner's
// other half), then the four quads summed by row rotations of 4 and 8 lanes.
__device__ __forceinline__ float row_reduce_scatter4(const float (&p)[4], int lane) {
    const bool o1 = lane & 1, o2 = lane & 2;
    float k0 = o1 ? p[1] : p[0], g0 = o1 ? p[0] : p[1];
    float k1 = o1 ? p[3] : p[2], g1 = o1 ? p[2] : p[3];
    k0 += WRNN_DPP(g0, 0xB1);            // quad_perm [1,0,3,2]: partner l^1
    k1 += WRNN_DPP(g1, 0xB1);
    float k = o2 ? k1 : k0, g = o2 ? k0 : k1;
    k += WRNN_DPP(g, 0x4E);              // quad_perm [2,3,0,1]: partner l^2
    k += WRNN_DPP(k, 0x124);             // row_ror:4
    k += WRNN_DPP(k, 0x128);             // row_ror:8
    return k;
}

// Register-blocked 16-lane dot engine: out[i] = W_i · X_{li & 3} for NW weight rows (W + i·ws)
// and 4 activation rows (X + j·xs; rows j >= nx re-read row 0: lanes with (li & 3) >= nx hold
// garbage), K4 float4 chunks split over the 16 lanes of a DPP row (lane li takes chunks li,
// li+16, …).  Each chunk load feeds 4·NW·4 FMAs, so LDS traffic per FMA is (NW + 4) / (4·NW) of
// a plain dot's.  KI > 0 fixes the per-lane chunk count (K4 = 16·KI) at compile time: the loop
// unrolls fully and the loads of later chunks are issued ahead of the FMAs of earlier ones
// (with a runtime count hipcc keeps load → lgkmcnt(0) → FMA per chunk).
template <int NW, int KI = 0>
__device__ __forceinline__ void bdot4(const float *__restrict__ W, int ws, const float *__restrict__ X, int xs, int nx,
                                      int K4, int li, float (&out)[NW]) {
    // packed fp32 FMAs (v_pk_fma_f32: two lanes of work per instruction, the fp32 vector peak):
    // each (weight row, activation row) pair keeps an even-k and an odd-k partial sum, added at
    // the end — the float4 halves .xy / .zw are already aligned register pairs, so no moves
    constexpr int NX = 4;
    const f4v *w4[NW];
    const f4v *x4[NX];
#pragma unroll
    for (int i = 0; i < NW; ++i) w4[i] = reinterpret_cast<const f4v *>(W + i * ws) + li;
#pragma unroll
    for (int j = 0; j < NX; ++j) x4[j] = reinterpret_cast<const f4v *>(X + (j < nx ? j : 0) * xs) + li;
    f2v acc[NW][NX];
#pragma unroll
    for (int i = 0; i < NW; ++i)
#pragma unroll
        for (int j = 0; j < NX; ++j) acc[i][j] = f2v{0.0f, 0.0f};
    auto step = [&](int k) {
        f4v wv[NW], xv[NX];
#pragma unroll
        for (int i = 0; i < NW; ++i) wv[i] = w4[i][16 * k];
#pragma unroll
        for (int j = 0; j < NX; ++j) xv[j] = x4[j][16 * k];
#pragma unroll
        for (int i = 0; i < NW; ++i)
#pragma unroll
            for (int j = 0; j < NX; ++j) {
                acc[i][j] = __builtin_elementwise_fma(wv[i].xy, xv[j].xy, acc[i][j]);
                acc[i][j] = __builtin_elementwise_fma(wv[i].zw, xv[j].zw, acc[i][j]);
            }
    };
    if (KI > 0) {
#pragma unroll
        for (int k = 0; k < KI; ++k) step(k);
    } else {
        for (int k = 0; 16 * k + li < K4; ++k) step(k);
    }
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        float p[NX];
#pragma unroll
        for (int j = 0; j < NX; ++j) p[j] = acc[i][j].x + acc[i][j].y;
        out[i] = row_reduce_scatter4(p, li);
    }
}

// Block-sparse gate rows of one 4-unit block-row: out[g] (lane li) = Σ_k blk[g][k] · x[4·col[g][k] …]
// for unit li & 3, gates g = 0..2.  Lanes of the 16-lane engine split the nonzero blocks; the
// four unit rows of each block are reduce-scattered so lane li ends up with unit li & 3.
__device__ __forceinline__ void sparse_gates4(const float *__restrict__ blk, const int *__restrict__ col,
                                              const int *__restrict__ cnt, int nbmax, const float *__restrict__ x,
                                              int li, float (&out)[3]) {
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        const float4 *b4 = reinterpret_cast<const float4 *>(blk + (size_t)g * nbmax * 16);
        const int *cg = col + g * nbmax;
        for (int k = li; k < cnt[g]; k += 16) {
            const float4 xv = *reinterpret_cast<const float4 *>(x + 4 * cg[k]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 wv = b4[4 * k + r];
                float a = p[r];
                a = fmaf(wv.x, xv.x, a);
                a = fmaf(wv.y, xv.y, a);
                a = fmaf(wv.z, xv.z, a);
                a = fmaf(wv.w, xv.w, a);
                p[r] = a;
            }
        }
        out[g] = row_reduce_scatter4(p, li);
    }
}

// ----------------------------------------------------------------------------- samplers
// One wave samples one row; the result is wave-uniform.
//
// MoL (utils/distribution.py:87-123): l = 30 logits [logit_probs | means | log_scales];
// u[k < 10] = log(-log(u1_k)) and u[10] = log(u2) - log(1 - u2), prepared off the critical path.
__device__ __forceinline__ float mol_sample(const float *l, const float *u, int lane) {
    float v = -INFINITY;
    if (lane < 10) v = l[lane] - u[lane];
    int k = 0;
    float best = lane_bcast(v, 0);
#pragma unroll
    for (int j = 1; j < 10; ++j) {
        const float vj = lane_bcast(v, j);
        if (vj > best) { best = vj; k = j; }
    }
    const float mean = l[10 + k];
    const float ls = fmaxf(l[20 + k], -32.23619130191664f);
    float x = mean + expf(ls) * u[10];
    x = x < -1.0f ? -1.0f : x;
    x = x > 1.0f ? 1.0f : x;
    return x;
}

// The same sampler with the logits in registers: lane l holds logit (l & 31) (lanes 0..29 are
// read), ul = u[lane] for lanes 0..9, u10 = u[10].  The argmax over lanes 0..9 runs in DPP
// row 0 (ties → the smaller index, as mol_sample's first-max scan); same arithmetic.
__device__ __forceinline__ float mol_sample_reg(float s, float ul, float u10, int lane) {
    float v = lane < 10 ? s - ul : -INFINITY;
    int i = lane;
#define WRNN_AM_STAGE(ctrl)                                                           \
    {                                                                                 \
        float ov = WRNN_DPP(v, ctrl);                                                 \
        int oi = __builtin_amdgcn_mov_dpp(i, (ctrl), 0xF, 0xF, false);                \
        am_merge(v, i, ov, oi);                                                       \
    }
    WRNN_AM_STAGE(0xB1) WRNN_AM_STAGE(0x4E) WRNN_AM_STAGE(0x141) WRNN_AM_STAGE(0x140)
#undef WRNN_AM_STAGE
    const int k = __builtin_amdgcn_readlane(i, 0);
    const float mean = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s), 10 + k));
    const float ls = fmaxf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s), 20 + k)),
                           -32.23619130191664f);
    float x = mean + expf(ls) * u10;
    x = x < -1.0f ? -1.0f : x;
    x = x > 1.0f ? 1.0f : x;
    return x;
}

// RAW (fatchord_version.py:231-237): softmax → Categorical (probs renormalised) → argmax(p / q),
// q ~ Exp(1) (the multinomial sampling path Categorical.sample() takes).  Returns the label.
template <int kClsPerLane>
__device__ __forceinline__ int raw_sample(const float *l, const float *u, int NC, int lane) {
    float e[kClsPerLane];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < kClsPerLane; ++k) {
        const int c = lane + 64 * k;
        e[k] = (c < NC) ? l[c] : -INFINITY;
        m = fmaxf(m, e[k]);
    }
    m = wave_max(m);
    float s1 = 0.0f;
#pragma unroll
    for (int k = 0; k < kClsPerLane; ++k) {
        const int c = lane + 64 * k;
        e[k] = (c < NC) ? expf(e[k] - m) : 0.0f;
        s1 += e[k];
    }
    s1 = wave_sum(s1);
    float s2 = 0.0f;
#pragma unroll
    for (int k = 0; k < kClsPerLane; ++k) {
        e[k] = e[k] / s1;
        s2 += e[k];
    }
    s2 = wave_sum(s2);
    float bv = -INFINITY;
    int bi = 0x7FFFFFFF;
#pragma unroll
    for (int k = 0; k < kClsPerLane; ++k) {
        const int c = lane + 64 * k;
        if (c < NC) am_merge(bv, bi, (e[k] / s2) / u[c], c);
    }
    return wave_argmax(bv, bi);
}

// The same for any class count (bits > 9, quantisation > 256): the exponentials are recomputed in
// each pass instead of held in registers — the same fp32 values in the same per-lane order, so
// the same label as raw_sample for NC <= 64·kClsPerLane.
__device__ __forceinline__ int raw_sample_any(const float *l, const float *u, int NC, int lane) {
    float m = -INFINITY;
    for (int c = lane; c < NC; c += 64) m = fmaxf(m, l[c]);
    m = wave_max(m);
    float s1 = 0.0f;
    for (int c = lane; c < NC; c += 64) s1 += expf(l[c] - m);
    s1 = wave_sum(s1);
    float s2 = 0.0f;
    for (int c = lane; c < NC; c += 64) s2 += expf(l[c] - m) / s1;
    s2 = wave_sum(s2);
    float bv = -INFINITY;
    int bi = 0x7FFFFFFF;
    for (int c = lane; c < NC; c += 64) am_merge(bv, bi, ((expf(l[c] - m) / s1) / s2) / u[c], c);
    return wave_argmax(bv, bi);
}

// RAW label → sample value (fatchord_version.py:235), fp32 like the reference
__device__ __forceinline__ float label_to_x(int label, int NC) { return (2.0f * (float)label) / ((float)NC - 1.0f) - 1.0f; }

// MoL sampler terms from the uniform draws (same fp32 operations as at sampling time)
__device__ __forceinline__ float mol_noise_term(float uu, int k) {
    return k < 10 ? logf(-logf(uu)) : (logf(uu) - logf(1.0f - uu));
}

__device__ __forceinline__ float gru_gate_math(float gi_r, float gi_z, float gi_n, float gh_r, float gh_z,
                                               float gh_n, float h_old) {
    // ATen gru_cell order (bit-exact vs torch.nn.GRUCell on CPU in the oracle):
    // r = σ(hr + ir), z = σ(hz + iz), n = tanh(in + hn·r), h' = (h − n)·z + n
    const float r = sigmoid_(gh_r + gi_r);
    const float z = sigmoid_(gh_z + gi_z);
    const float n = tanh_(gi_n + gh_n * r);
    return (h_old - n) * z + n;
}

// LDS-only workgroup barrier.  Unlike __syncthreads() it does not drain vmcnt, so the loader
// wave's LDS-DMA and the publishers' granule stores stay in flight across it.
__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}


#define WRNN_GPTR(p) ((__attribute__((address_space(1))) void *)(p))
#define WRNN_LPTR(p) ((__attribute__((address_space(3))) void *)(p))

}  // namespace wrnn
