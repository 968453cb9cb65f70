// fatchord_xcds.hip — XCD-resident persistent kernel for MoL rows with rnn 896 and 4×4
// block-sparse GRU matrices (BASELINE config 4; weights pruned by pruning.py): the sample loop of
// models/fatchord_version.py:201-241 for ONE row on the 32 CUs of ONE XCD, up to eight rows (one
// per XCD) per launch.  Same scheme as fatchord_xcd.hip (dense rnn 512; read its header first):
// XCD membership from HW_REG_XCC_ID, plain-store granule hand-offs that stay in the XCD's L2,
// 16-byte sc1 polls, GRU1 for all units in every workgroup (rank-1 in x), fc1 / fc2 in the
// registers of the waves that poll their inputs, LDS step flags that keep the off-critical
// traffic out of the critical hop windows.
//
// Workgroup c owns GRU units 28c..28c+27 = seven 4-unit block-rows ub per gate, and fc rows
// 16c..16c+15.  The GRU matrices are held as their nonzero 4×4 blocks, at most 32 per gate
// block-row: a 16-lane "engine" computes one block-row, lane li the blocks li and li + 16
// (4×4 block · the 4 activations at its column block, read from LDS), then Σ over the engine.
//   B1 → GRU1 for all 896 units (threads tid and tid + 512) from the gathered terms S
//   B2 → GRU2: wave ub (0..6), engine q (0..2) = gate q of block-row ub (W_ih2 blocks in VGPRs);
//        permlane swaps bring the z and n sums to engine 0, whose lanes 0..3 finish units 4ub + l
//        and publish y = x_I + h1 + h2                                             [hop Y]
//   waves 4..7 poll y (7 × 16 B per lane) → fc1 rows 4h.. (h = w − 4) in registers → relu [hop F1]
//   waves 0..3 poll f1 → fc2 rows 4w.. → relu → fc3 partials; waves 1..3 → wave 0   [hop F2]
//   wave 0 polls the 32 × 32 partials → Σ + b3 → MoL sample (redundant, bit-identical) → x_t
// Four rows per fc wave (round 5; eight on two waves before: fc1's 8 × 7 weight pairs per lane
// spilled 28 VGPRs).  Off the critical path, in each wave's idle windows: waves 0..3 (idle from
// GRU2 until f1 arrives) W_hh1·h1 (LDS blocks, one engine per gate block-row, 21 = 16 + 5) → the
// GRU1 terms of step t+1, published after "y gathered", and h2; waves 1..3 after their fc3
// hand-off and wave 6 the four quarters of the next S (round 5: on waves 4..7 before, which then
// arrived last at the step-end barrier: 3.63 → 3.42 µs/step); waves 4..7 (idle from their f1
// publish to the step's end) h2 out, after "f1 gathered": the h2 gather (wave 4), the ring
// (wave 7), then W_hh2·h2 (LDS blocks, 16 + 5 engines).  fp32, sums re-associated
// (tolerance-checked).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fatchord_loop.h"
#include "fatchord_xcds.h"
#include "wrnn_device.h"
#include "xcd_device.h"

namespace wrnn {

#ifndef WRNN_XCDS_DIAG
#define WRNN_XCDS_DIAG 0   // timing diagnostics (wrong results): 1 skip the S gathers, 2 skip the h2 gather
#endif
#ifndef WRNN_XCDS_RS
#define WRNN_XCDS_RS 1   // block-row sums reduce-scattered over the engine (0: four row sums + select, A/B)
#endif
#ifndef WRNN_XCDS_GRU2_STAMPS
#define WRNN_XCDS_GRU2_STAMPS 0   // diagnostics: stamps 12..14 inside GRU2 (wave 0) instead of the ring / GH2 ones
#endif

// 8 rows of an (NK·128)-wide layer against a vector polled into registers by ONE wave: lane l
// holds the pairs k = 0..NK-1 at granules 2(l + 64k) + {0, 1} (xk[k]) and the matching weights
// of row r in w[r·NK + k].  Packed FMAs, then the reduce-scatter of fc8_rows: o[j] = full sum of
// row j + 2·(l >> 4), identical bits in all 16 lanes of DPP row l >> 4.
template <int NK>
__device__ __forceinline__ void fc8_rows_k(const f2v *w, const f2v (&xk)[NK], float (&o)[2]) {
    float s[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        f2v a = __builtin_elementwise_fma(w[r * NK], xk[0], f2v{0.0f, 0.0f});
        f2v b = __builtin_elementwise_fma(w[r * NK + 1], xk[1], f2v{0.0f, 0.0f});
#pragma unroll
        for (int k = 2; k < NK; k += 2) a = __builtin_elementwise_fma(w[r * NK + k], xk[k], a);
#pragma unroll
        for (int k = 3; k < NK; k += 2) b = __builtin_elementwise_fma(w[r * NK + k], xk[k], b);
        const f2v t = a + b;
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

// 4 rows of an (NK·128)-wide layer against a vector polled into registers by ONE wave (lane l:
// pairs k at granules 2(l + 64k) + {0, 1}, weights of row r in w[r·NK + k]).  Packed FMAs, then a
// reduce-scatter — permlane32 swap (row r vs r + 2), permlane16 swap (r vs r + 1), DPP sum over
// the 16 lanes of a row — leaves the full sum of row l >> 4, identical bits in the 16 lanes of
// DPP row l >> 4.
template <int NK>
__device__ __forceinline__ float fc4_rows_k(const f2v *w, const f2v (&xk)[NK]) {
    float s[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        f2v a = __builtin_elementwise_fma(w[r * NK], xk[0], f2v{0.0f, 0.0f});
        f2v b = __builtin_elementwise_fma(w[r * NK + 1], xk[1], f2v{0.0f, 0.0f});
#pragma unroll
        for (int k = 2; k < NK; k += 2) a = __builtin_elementwise_fma(w[r * NK + k], xk[k], a);
#pragma unroll
        for (int k = 3; k < NK; k += 2) b = __builtin_elementwise_fma(w[r * NK + k], xk[k], b);
        const f2v t = a + b;
        s[r] = t.x + t.y;
    }
    float h[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {   // lanes < 32 keep row j, lanes ≥ 32 row j + 2
        const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s[j]), __float_as_uint(s[j + 2]), false, false);
        h[j] = __uint_as_float(q[0]) + __uint_as_float(q[1]);
    }
    // even DPP rows keep h[0], odd rows h[1]: DPP row g ends with row g
    const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(h[0]), __float_as_uint(h[1]), false, false);
    return row_sum16(__uint_as_float(q[0]) + __uint_as_float(q[1]));
}

// g[i] for a per-lane i in 0..3 as three v_cndmask (the nested ?: form compiled into exec-mask
// branches: ≈ 30 scalar / branch instructions per call in the GRU2 epilogue)
__device__ __forceinline__ float sel4(const float (&g)[4], int i) {
    const float a = (i & 1) ? g[1] : g[0];
    const float b = (i & 1) ? g[3] : g[2];
    return (i & 2) ? b : a;
}

// One gate block-row on a 16-lane engine: Σ over its nonzero 4×4 blocks of W_blk · v[4j..4j+3];
// this lane holds blocks wa (column block ja) and wb (jb), rows as float4.  Returns, in lane l,
// the full sum of row l & 3 (every consumer takes that row: the GRU2 epilogue, the term and
// W_hh2·h2 stores of lanes li < 4).
__device__ __forceinline__ float sp_block_row(const f4v (&wa)[4], const f4v (&wb)[4], int ja, int jb,
                                              const float *v, int lane) {
    const f4v xa = lds4(v + 4 * ja), xb = lds4(v + 4 * jb);
    float t[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        f2v acc = __builtin_elementwise_fma(wa[r].xy, xa.xy, f2v{0.0f, 0.0f});
        f2v acc2 = __builtin_elementwise_fma(wa[r].zw, xa.zw, f2v{0.0f, 0.0f});
        acc = __builtin_elementwise_fma(wb[r].xy, xb.xy, acc);
        acc2 = __builtin_elementwise_fma(wb[r].zw, xb.zw, acc2);
        const f2v tt = acc + acc2;
        t[r] = tt.x + tt.y;
    }
#if WRNN_XCDS_RS
    // reduce-scatter over the engine's 16 lanes: lane l keeps rows of its parity (l & 1) against
    // lane l ^ 1, then row l & 3 against l ^ 2, then sums the four lanes of its residue class
    // (row_ror 4, 8): 5 DPP adds and 6 selects on a 4-deep chain instead of four 4-deep row sums
    const bool odd = (lane & 1) != 0, hi = (lane & 2) != 0;
    const float u0 = odd ? t[1] : t[0], v0 = odd ? t[0] : t[1];
    const float u1 = odd ? t[3] : t[2], v1 = odd ? t[2] : t[3];
    const float a0 = u0 + WRNN_DPP(v0, 0xB1), a1 = u1 + WRNN_DPP(v1, 0xB1);   // quad_perm [1,0,3,2]
    const float keep = hi ? a1 : a0, send = hi ? a0 : a1;
    float b = keep + WRNN_DPP(send, 0x4E);                                     // quad_perm [2,3,0,1]
    b += WRNN_DPP(b, 0x124);                                                   // row_ror:4
    b += WRNN_DPP(b, 0x128);                                                   // row_ror:8
    return b;
#else
    float g[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) g[r] = row_sum16(t[r]);
    return sel4(g, lane & 3);
#endif
}

#ifndef WRNN_XCDS_SQ_EARLY
#define WRNN_XCDS_SQ_EARLY 1   // S quarters on waves 1, 3, 6, 2 (0: on the fc1 waves 4..7, A/B)
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
__global__ __launch_bounds__(kXThreads, 2) void fatchord_xcds_kernel(XcdsArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int R = kSR, TW = kXcdWgs * kSTerms;
    const XcdsLds ll = xcds_lds_layout();
    const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, eng = lane >> 4;
    // the wave index wave-uniform (SGPR): its role branches become scalar, its offsets scalar operands
    const int wave = WRNN_XCD_UNIFORM_WAVE ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
    float *h1s = smem + ll.h1, *h2s = smem + ll.h2, *sg = smem + ll.sg, *w3s = smem + ll.w3, *f2x = smem + ll.f2x;
    float *ring = smem + ll.ring, *nzr = smem + ll.nz, *gh2s = smem + ll.gh2, *cst = smem + ll.cst, *xs = smem + ll.xs;
    float *whh1b = smem + ll.whh1b, *whh2b = smem + ll.whh2b;
    const int *whh1c = reinterpret_cast<const int *>(smem + ll.whh1c), *whh2c = reinterpret_cast<const int *>(smem + ll.whh2c);
    int *misc = reinterpret_cast<int *>(smem + ll.misc);
    int *abort_flag = misc, *h2ready = misc + 2, *ygot = misc + 4, *f1got = misc + 5;
    int *const f2ready[3] = {misc + 3, misc + 6, misc + 7};   // fc2 waves 1..3: partials in f2x

    // ---- membership: XCD k (row b0 + k) and index c within it
    if (tid == 0) {
        const int k = (int)xcc_id();
        int c = kXcdWgs;
        if (k < a.nb) c = atomicAdd(&a.members[k], 1);
        misc[1] = (k < a.nb && c < kXcdWgs) ? k * kXcdWgs + c : -1;
        misc[0] = 0;
        for (int i = 2; i < 8; ++i) misc[i] = 0;
    }
    if (tid < 3 * 64) f2x[tid] = 0.0f;   // the fc3 hand-off pairs: tag 0, which no step carries
    __syncthreads();
    const int mem = __builtin_amdgcn_readfirstlane(misc[1]);   // wave-uniform: hop addresses in SGPRs
    if (mem < 0) return;
    const int k = mem / kXcdWgs, c = mem - k * kXcdWgs;
    const int b = a.b0 + k;
    const int t_end = a.t0 + a.Lc;
    const int t_terms = min(t_end, a.L - 1);
    unsigned long long *xg = a.xg + (size_t)k * kXXcdStride;
    auto XG = [&](int hop) { return xg + (size_t)hop * kXHopStride; };
    const __amdgpu_buffer_rsrc_t xgr = __builtin_amdgcn_make_buffer_rsrc(xg, 0, 0x7fffffff, 0x00020000);   // publishes
    auto XGI = [&](int hop) { return hop * (int)kXHopStride; };                                          // granule index
    auto RING = [&](int t) { return ring + (t & (kXRing - 1)) * kSTerms; };
    auto NZ = [&](int t) { return nzr + (t & (kXRing - 1)) * kXNoise; };
    auto TERMS = [&](int t) { return a.terms + ((size_t)(t - a.t0) * a.nb + k) * TW + (size_t)c * kSTerms; };
    const float *S = a.slab + (size_t)c * a.s.total;
    const unsigned long long prow = (unsigned long long)(a.row0 + k);

    // ---- register-resident weights
    //   wg (waves 0..6, engines 0..2): the two W_ih2 blocks of this lane in gate block-row
    //     (q = engine, ub = wave), columns ja / jb
    //   wr (one register set, by role): waves 4..7: fc1 rows 4h + r (h = w − 4) at the y granules
    //     this lane polls (r·7 + k); waves 0..3: fc2 rows 4w + r (r·4 + k); wave 0: the F2 poll
    //     buffer in wr[16..31]
    f4v wg[8];
    // 16-byte aligned: wave 0 reuses wr[16..31] as its F2 poll buffer (eight u4v)
    alignas(16) f2v wr[32];
    constexpr int kFc2Pairs = 4 * (512 / 128);   // fc2: 4 rows x 512 / (64 lanes x 2) pairs per lane
    static_assert(kFc2Pairs <= 16, "wave 0's fc2 weights must fit wr[0..15]: wr[16..31] is its F2 poll buffer");
    static_assert(4 * kSPairs <= 32, "fc1 rows of a wave must fit wr[]");
    static_assert(sizeof(f2v) * 16 == 8 * sizeof(u4v), "the F2 poll buffer is eight 16-byte loads");
    int ja = 0, jb = 0;
    {
        const bool gw = wave < kSUB && eng < 3;
        const int br = eng * kSUB + wave;
        const float *blk = S + a.s.wih2b + ((size_t)br * kSNB + li) * 16;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            wg[i] = gw ? *reinterpret_cast<const f4v *>(blk + 4 * i) : f4v{0.0f, 0.0f, 0.0f, 0.0f};
            wg[4 + i] = gw ? *reinterpret_cast<const f4v *>(blk + 16 * 16 + 4 * i) : f4v{0.0f, 0.0f, 0.0f, 0.0f};
        }
        if (gw) {
            const int *cc = reinterpret_cast<const int *>(S + a.s.wih2c) + br * kSNB;
            ja = cc[li];
            jb = cc[li + 16];
        }
    }
    if (wave >= 4) {
        const float *W = S + a.s.w1 + (wave - 4) * 4 * R;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int r = i / kSPairs, kk = i - r * kSPairs;
            wr[i] = i < 4 * kSPairs ? *reinterpret_cast<const f2v *>(W + r * R + 2 * (lane + 64 * kk)) : f2v{0.0f, 0.0f};
        }
    } else {
        const float *W = S + a.s.w2 + wave * 4 * 512;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int r = i >> 2, kk = i & 3;
            wr[i] = i < kFc2Pairs ? *reinterpret_cast<const f2v *>(W + r * 512 + 2 * (lane + 64 * kk)) : f2v{0.0f, 0.0f};
        }
    }
    // GRU1 of units tid and tid + 512 (tid < 384): x-coefficients
    const bool two = tid + 512 < R;
    const int u2 = two ? tid + 512 : tid;
    const float q1r = S[a.s.q1a + tid], q1z = S[a.s.q1a + R + tid], q1n = S[a.s.q1a + 2 * R + tid];
    const float q1r2 = S[a.s.q1a + u2], q1z2 = S[a.s.q1a + R + u2], q1n2 = S[a.s.q1a + 2 * R + u2];
    // GRU2 unit of lanes 0..3 of waves 0..6 (engine 0)
    const int ul = min(4 * wave + (lane & 3), kSU - 1);

    // sampler noise of step t → NZ(t): u1 → log(-log u1) (distribution.py:107), u2 → log u2 − log(1 − u2) (:119)
    auto noise_term = [&](int t) -> float {
        float uu;
        if (a.noise) uu = a.noise[((size_t)t * a.Bt + b) * 11 + lane];
        else uu = philox_noise(a.seed, prow, (uint32_t)t, (uint32_t)lane, 1);
        return mol_noise_term(uu, lane);
    };
    // GRU1 term(s) of step t for row rr (u·3 + q):
    //   q = 0: S_r = (GH1_r + b_hh,r) + (P1_r + b_ih,r), q = 1: S_z likewise,
    //   q = 2: Gh_n = GH1_n + b_hh,n (term 3) and Gi_n = P1_n + b_ih,n (term 2)
    auto publish_term = [&](int t, int rr, float gh) {
        const int u = rr / 3, q = rr - 3 * u;
        const float p1 = RING(t)[SX_P1 + rr], bh = cst[SC_BHH1 + rr], bi = cst[SC_BIH1 + rr];
        const int g = XGI(XH_S0 + (t & 1)) + (c * kSU + u) * 4;
        const uint32_t tag = (uint32_t)t + 1u;
        if (q < 2) {
            xpub_b(xgr, g + q, tag, (gh + bh) + (p1 + bi));
        } else {
            xpub_b(xgr, g + 3, tag, gh + bh);
            xpub_b(xgr, g + 2, tag, p1 + bi);
        }
    };
    // a gate block-row of W_hh1 / W_hh2 from LDS (block-row br of this engine)
    auto lds_block_row = [&](const float *wb, const int *wc, int br, const float *v) -> float {
        const float *p = wb + ((size_t)br * kSNB + li) * 16;
        f4v wa4[4], wb4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            wa4[i] = lds4(p + 4 * i);
            wb4[i] = lds4(p + 16 * 16 + 4 * i);
        }
        return sp_block_row(wa4, wb4, wc[br * kSNB + li], wc[br * kSNB + li + 16], v, lane);
    };
    // The 21 gate block-rows of W_hh1 / W_hh2 on a wave quad's 16 engines: pass 0 block-row 4·(w & 3) + e,
    // pass 1 block-rows 16..20 on the first wave of the quad (engines 0..3) and the second (engine 0).
    // W_hh1·h1 → GRU1 terms of step t+1 on waves 0..3, W_hh2·h2 → gh2s on waves 4..7.
    const int wq = wave & 3;
    const int br0 = 4 * wq + eng, br1 = wq == 0 ? 16 + eng : (wq == 1 && eng == 0) ? 20 : -1;
    auto gh_dots = [&](const float *wbk, const int *wck, const float *v, int br) -> float {
        return lds_block_row(wbk, wck, br >= 0 ? br : 0, v);
    };
    auto publish_terms = [&](int t, int br, float g) {   // g: row li & 3 of block-row br
        if (br >= 0 && li < 4) {
            const int q = br / kSUB, ub = br - q * kSUB;
            publish_term(t, (4 * ub + li) * 3 + q, g);
        }
    };
    auto gh2_dots = [&](int br) {
        const float g = gh_dots(whh2b, whh2c, h2s, br);
        if (br >= 0 && li < 4) {
            const int q = br / kSUB, ub = br - q * kSUB;
            gh2s[(4 * ub + li) * 3 + q] = g;
        }
    };
    // a quarter of step t's GRU1 terms (896 granules each, one poll round): waves 1, 3, 6, 2
    // (quarters 0..3; fc2 waves 1..3 are idle after their fc3 hand-off, the fc1 waves were the last
    // at the step-end barrier) — WRNN_XCDS_SQ_EARLY 0: waves 4..7
    auto sq_of = [&](int w) { return WRNN_XCDS_SQ_EARLY ? (w == 1 ? 0 : w == 3 ? 1 : w == 6 ? 2 : w == 2 ? 3 : -1) : w - 4; };
    auto gather_terms = [&](int t) {
        if (WRNN_XCDS_DIAG & 1) return;
        const int qq = sq_of(wave);
        xgather16<kSPairs>(XG(XH_S0 + (t & 1)) + qq * R, (uint32_t)t + 1u, a.ctl, a.timeout_ticks, t,
                           XH_S0 + (t & 1), abort_flag, lane, [&](int i, float v0, float v1) {
                               *reinterpret_cast<f2v *>(sg + qq * R + i) = f2v{v0, v1};
                           });
    };
    auto set_flag = [&](int *f, uint32_t tag) {
        if (lane == 0) __hip_atomic_store(f, (int)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto wait_flag = [&](int *f, uint32_t tag) {
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)tag)
            __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
    };

    // ---- prologue: W_hh1 / W_hh2 blocks, fc3 columns, small vectors, ring slots t0..t0+2, state
    {
        constexpr int NBF = kSBR * kSNB * 16 / 4;   // float4s per block matrix
        const f4v *s1 = reinterpret_cast<const f4v *>(S + a.s.whh1b), *s2 = reinterpret_cast<const f4v *>(S + a.s.whh2b);
        f4v *d1 = reinterpret_cast<f4v *>(whh1b), *d2 = reinterpret_cast<f4v *>(whh2b);
        for (int i = tid; i < NBF; i += kXThreads) {
            d1[i] = s1[i];
            d2[i] = s2[i];
        }
        for (int i = tid; i < kSBR * kSNB; i += kXThreads) {
            smem[ll.whh1c + i] = S[a.s.whh1c + i];
            smem[ll.whh2c + i] = S[a.s.whh2c + i];
        }
        for (int i = tid; i < kXFcRows * 32; i += kXThreads) w3s[i] = S[a.s.w3 + i];
        for (int i = tid; i < kSCst; i += kXThreads) cst[i] = S[a.s.cst + i];
        for (int t = a.t0; t < a.t0 + 3; ++t) {
            if (t <= t_terms)
                for (int i = tid; i < kSTerms; i += kXThreads) RING(t)[i] = TERMS(t)[i];
            if (wave == 1 && lane < 11 && t < a.L) NZ(t)[lane] = noise_term(t);
        }
    }
    // wave 7 stages the ring entries of a step in wg (its GRU2 registers, unused by wave 7):
    // conditioning terms (lanes < 57, one float4 each) and the injected sampler noise (lanes < 11)
    auto stage_ring = [&](int t) {
        if (t <= t_terms && lane < kSTerms / 4) wg[0] = reinterpret_cast<const f4v *>(TERMS(t))[lane];
        if (a.noise && t < a.L && lane < 11) wg[1].x = a.noise[((size_t)t * a.Bt + b) * 11 + lane];
    };
    if (wave == 7) stage_ring(a.t0 + 3);
    const bool resume = a.t0 > 0;
    float *st = a.state + ((size_t)k * kXcdWgs + c) * kSStateW;
    constexpr int oSG = kSR, oGH2 = kSR + 4 * kSR, oH2 = oGH2 + 84, oX = oH2 + kSU;
    float h1v = resume ? st[tid] : 0.0f;               // h1 of units tid, tid + 512 (this thread)
    float h1v2 = (resume && two) ? st[u2] : 0.0f;
    float h2own = resume ? st[oH2 + ul] : 0.0f;       // h2 of unit ul (lanes 0..3 of waves 0..6)
    if (resume) {
        for (int i = tid; i < 4 * R; i += kXThreads) sg[i] = st[oSG + i];
        if (tid < 84) gh2s[tid] = st[oGH2 + tid];
        if (tid == 0) xs[(a.t0 + 1) & 1] = st[oX];
    } else {
        if (tid < 84) gh2s[tid] = 0.0f;
        if (tid == 0) xs[1] = 0.0f;
    }
    __syncthreads();
    if (!resume) {   // GRU1 terms of step 0 (GH1 = 0), published and gathered
        if (wave < 4) {
            publish_terms(0, br0, 0.0f);
            publish_terms(0, br1, 0.0f);
        }
        if (sq_of(wave) >= 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            gather_terms(0);
        }
    }
    __syncthreads();
    if (*abort_flag) return;

    float x = xs[(a.t0 + 1) & 1];                    // x_{t-1}, wave-uniform
    f4v s4 = lds4(sg + 4 * tid), s4b = lds4(sg + 4 * u2);
    for (int t = a.t0; t < t_end; ++t) {
        const uint32_t tag = (uint32_t)t + 1u;
        const bool more = t + 1 < a.L;
        const float *tr = RING(t);
        XSTAMP(0);
        // operands of the GRU2 gate math (unit ul), read before GRU1
        float q2v[3], p2v[3], bi2[3], ghv[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            q2v[q] = cst[SC_Q2 + ul * 3 + q];
            p2v[q] = tr[SX_P2 + ul * 3 + q];
            bi2[q] = cst[SC_BIH2 + ul * 3 + q];
            ghv[q] = gh2s[ul * 3 + q] + cst[SC_BHH2 + ul * 3 + q];
        }
        const float wi0v = cst[SC_WI0 + ul], civ = tr[SX_CI + ul];
        // ---- GRU1 (:208-210), units tid and tid + 512
        {
            const float r = sigmoid_(fmaf(x, q1r, s4.x));
            const float z = sigmoid_(fmaf(x, q1z, s4.y));
            const float n = tanh_(fmaf(x, q1n, s4.z) + s4.w * r);
            h1v = (h1v - n) * z + n;
            h1s[tid] = h1v;
            if (two) {
                const float r2 = sigmoid_(fmaf(x, q1r2, s4b.x));
                const float z2 = sigmoid_(fmaf(x, q1z2, s4b.y));
                const float n2 = tanh_(fmaf(x, q1n2, s4b.z) + s4b.w * r2);
                h1v2 = (h1v2 - n2) * z2 + n2;
                h1s[u2] = h1v2;
            }
        }
        float p2q[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) p2q[q] = fmaf(x, q2v[q], p2v[q]) + bi2[q];
        const float xi = fmaf(wi0v, x, civ);   // x_I of unit ul
        bar();
        XSTAMP(1);
        // ---- GRU2 (:212-214): engine q of wave ub → gate q of units 4ub..4ub+3 (W_ih2[:, :R]·h1)
        if (wave < kSUB) {
            // x_I + h1 of unit 4ub + (lane & 3) (:212) before the dots, pinned there (hipcc sinks the
            // h1 LDS read into the publishing lanes' branch after the gate math otherwise)
            float yb = xi + h1s[c * kSU + ul];
            asm volatile("" : "+v"(yb));
            const float gs = sp_block_row(*reinterpret_cast<const f4v(*)[4]>(&wg[0]),
                                          *reinterpret_cast<const f4v(*)[4]>(&wg[4]), ja, jb, h1s, lane);
            if (WRNN_XCDS_GRU2_STAMPS) {
                asm volatile("" ::"v"(gs));
                XSTAMP(12);
            }
            // every lane keeps its row (lane & 3) of its engine's gate; engine 0 collects z (engine 1,
            // one permlane16 swap) and n (engine 2, one permlane32 swap) — lane l < 4 then holds
            // r, z, n of unit 4ub + l (two swaps instead of one per row and gate)
            const float gz = __uint_as_float(
                __builtin_amdgcn_permlane16_swap(__float_as_uint(gs), __float_as_uint(gs), false, false)[1]);
            const float gn = __uint_as_float(
                __builtin_amdgcn_permlane32_swap(__float_as_uint(gs), __float_as_uint(gs), false, false)[1]);
            if (WRNN_XCDS_GRU2_STAMPS) {
                asm volatile("" ::"v"(gz), "v"(gn));
                XSTAMP(13);
            }
            const float hn = gru_gate_math(gs + p2q[0], gz + p2q[1], gn + p2q[2], ghv[0], ghv[1], ghv[2], h2own);
            h2own = hn;
            if (WRNN_XCDS_GRU2_STAMPS) {
                asm volatile("" ::"v"(hn));
                XSTAMP(14);
            }
            // y = (x_I + h1) + h2 (:212, :216)
            const float y = yb + hn;
            if (lane < 4) xpub_b(xgr, XGI(XH_Y) + c * kSU + ul, tag, y);
        }
        XSTAMP(2);
        auto pub_h2 = [&]() {
            if (wave < kSUB && lane < 4) xpub_b(xgr, XGI(XH_H2) + c * kSU + ul, tag, h2own);
        };
        // fc waves: lane l ends fc4_rows_k with row 4h + (l >> 4); lanes with (l & 15) == 0 publish it
        const int rq = lane >> 4;
        if (wave < 4) {
            // ---- waves 0..3: W_hh1·h1 (GRU1 terms of step t+1) in hop Y's window, published after
            // y gathered with h2; then hop F1 → fc2 (:220-221) rows 4w.. → relu → fc3 partial logits
            // of those rows (:223); waves 1..3 hand theirs to wave 0 (LDS, flags), wave 0 publishes
            // the workgroup's line (hop F2), polls all 32 lines and samples
            if (more) {
                const float g0 = gh_dots(whh1b, whh1c, h1s, br0);
                const float g1 = wq < 2 ? gh_dots(whh1b, whh1c, h1s, br1) : 0.0f;
                wait_flag(ygot, tag);
                publish_terms(t + 1, br0, g0);
                if (wq < 2) publish_terms(t + 1, br1, g1);
                pub_h2();
                XSTAMPW(9, 1);
            }
            const float v2 = tr[SX_V2 + 4 * wave + rq];
            float w3c[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) w3c[r] = w3s[(4 * wave + r) * 32 + (lane & 31)];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u4v v[4];
            xpoll16<4>(XG(XH_F1), tag, a.ctl, a.timeout_ticks, t, XH_F1, abort_flag, lane, v);
            if (wave == 1) set_flag(f1got, tag);
            XSTAMPW(5, 1);
            f2v fk[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) fk[kk] = f2v{__uint_as_float(v[kk].x), __uint_as_float(v[kk].z)};
            const float f = fc4_rows_k<4>(wr, fk) + v2;
            const float f2 = f > 0.0f ? f : 0.0f;
            float p = 0.0f;
#pragma unroll
            for (int g = 0; g < 4; ++g) p = fmaf(w3c[g], lane_bcast(f2, 16 * g), p);
            // waves 1..3 → wave 0: 8-byte (value, tag) pairs in LDS, polled by wave 0's lanes
            // themselves (one LDS round trip less than data + flags + a flag poll)
            unsigned long long *f2p = reinterpret_cast<unsigned long long *>(f2x);
            if (wave != 0) {
                if (lane < 32)
                    __hip_atomic_store(f2p + (wave - 1) * 32 + lane, ((unsigned long long)tag << 32) | __float_as_uint(p),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (WRNN_XCDS_SQ_EARLY && more) {   // a quarter of the next S (hop F1 polled: its window is over)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    gather_terms(t + 1);
                }
            } else {
                // waves 1..3 store on every path (their polls are bounded); the abort word ends the
                // wait too should that ever change
                unsigned spin = 0;
                unsigned long long pv[3] = {(unsigned long long)tag << 32, (unsigned long long)tag << 32,
                                            (unsigned long long)tag << 32};
                for (;;) {
                    if (lane < 32) {
#pragma unroll
                        for (int w = 0; w < 3; ++w)
                            pv[w] = __hip_atomic_load(f2p + w * 32 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    const bool ok = ((uint32_t)(pv[0] >> 32) == tag) & ((uint32_t)(pv[1] >> 32) == tag) &
                                    ((uint32_t)(pv[2] >> 32) == tag);
                    if (__ballot(!ok) == 0) break;
                    if ((++spin & 255u) == 0 &&
                        __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                        break;
                }
                if (lane < kXF2Line)   // 30, 31: zero weights
                    xpub_b(xgr, XGI(XH_F2) + c * kXF2Line + lane, tag,
                           ((p + __uint_as_float((uint32_t)pv[0])) + __uint_as_float((uint32_t)pv[1])) +
                               __uint_as_float((uint32_t)pv[2]));
                XSTAMPW(6, 0);
                // ---- hop F2: Σ of the 32 workgroups' partials + b3 → sample
                const int jp = lane & 15, pg = lane >> 4;
                const float ua = NZ(t)[jp < 5 ? 2 * jp : 0], ub = NZ(t)[jp < 5 ? 2 * jp + 1 : 0], u10 = NZ(t)[10];
                const float b3a = cst[SC_B3 + 2 * jp], b3b = cst[SC_B3 + 2 * jp + 1];
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const __amdgpu_buffer_rsrc_t rf = hop_rsrc(XG(XH_F2));
                const int goff = pg * 8 * kXF2Line * 8 + jp * 16;
                const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
                unsigned spins = 0;
                u4v *vv = reinterpret_cast<u4v *>(&wr[16]);   // wave 0's fc2 weights are wr[0..15]
                for (;;) {   // one wave-uniform exit; the values taken after the loop
#pragma unroll
                    for (int m = 0; m < 8; ++m) vv[m] = ld16_sc1(rf, goff + m * kXF2Line * 8);
                    bool ok = true;
#pragma unroll
                    for (int m = 0; m < 8; ++m) ok &= (vv[m].y == tag) & (vv[m].w == tag);
                    if (__ballot(!ok) == 0) break;
                    if ((++spins & 63u) == 0) {
                        const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - c0) > a.timeout_ticks;
                        const bool other = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                        if (late || other) {
                            if (late) record_abort(a.ctl, -4, t, XH_F2, blockIdx.x);
                            *abort_flag = 1;
                            break;
                        }
                    }
                }
                float pa[8], pb[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    pa[m] = __uint_as_float(vv[m].x);
                    pb[m] = __uint_as_float(vv[m].z);
                }
                XSTAMP(7);
#pragma unroll
                for (int n = 4; n >= 1; n /= 2)
#pragma unroll
                    for (int m = 0; m < n; ++m) {
                        pa[m] += pa[m + n];
                        pb[m] += pb[m + n];
                    }
                cross_rows_pair(pa[0], pb[0]);
                const float la = pa[0] + b3a, lb = pb[0] + b3b;   // logits 2jp, 2jp+1
                x = mol_sample_pairs(la, lb, ua, ub, u10, jp);
                if (lane == 0) {
                    xs[t & 1] = x;
                    if (c == 0) a.out[(size_t)b * a.L + t] = x;
                }
                XSTAMP(8);
            }
        } else {
            // ---- waves 4..7: hop Y → fc1 (:216-218) rows 4h.. in registers → relu → hop F1
            const int hf = wave - 4, rg = 4 * hf + rq;
            const float v1 = tr[SX_V1 + rg];
            if (wave == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u4v v[kSPairs];
            xpoll16<kSPairs>(XG(XH_Y), tag, a.ctl, a.timeout_ticks, t, XH_Y, abort_flag, lane, v);
            if (hf == 0) set_flag(ygot, tag);
            // h2 out (waves 4..6 hold GRU2 units) before fc1: a store issued here lands in the fc1
            // compute, not in hop F1's window
            if (more) pub_h2();
            XSTAMPW(3, 4);
            f2v yk[kSPairs];
#pragma unroll
            for (int kk = 0; kk < kSPairs; ++kk) yk[kk] = f2v{__uint_as_float(v[kk].x), __uint_as_float(v[kk].z)};
            const float A = fc4_rows_k<kSPairs>(wr, yk) + v1;
            if ((lane & 15) == 0) xpub_b(xgr, XGI(XH_F1) + c * kXFcRows + rg, tag, A > 0.0f ? A : 0.0f);
            XSTAMPW(4, 4);
            if (more) {
                // after f1 gathered: h2 (wave 4, then its flag), an S quarter (wave 6; all four with
                // WRNN_XCDS_SQ_EARLY 0), the ring (wave 7: step t+3's entries from the registers
                // loaded a step ago, the load for t+4 lands during the next step); after h2
                // gathered: W_hh2·h2
                wait_flag(f1got, tag);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (wave == 4) {
                    if (!(WRNN_XCDS_DIAG & 2))
                        xgather16<kSPairs>(XG(XH_H2), tag, a.ctl, a.timeout_ticks, t, XH_H2, abort_flag, lane,
                                           [&](int i, float v0, float v1) { *reinterpret_cast<f2v *>(h2s + i) = f2v{v0, v1}; });
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    set_flag(h2ready, tag);
                    XSTAMPW(10, 4);
                }
                if (sq_of(wave) >= 0) gather_terms(t + 1);
                XSTAMPW(11, 5);
                if (wave == 7) {
                    if (t + 3 <= t_terms && lane < kSTerms / 4) reinterpret_cast<f4v *>(RING(t + 3))[lane] = wg[0];
                    if (t + 3 < a.L && lane < 11)
                        NZ(t + 3)[lane] = mol_noise_term(a.noise ? wg[1].x : philox_noise(a.seed, prow, (uint32_t)(t + 3), (uint32_t)lane, 1), lane);
                    stage_ring(t + 4);
                    if (!WRNN_XCDS_GRU2_STAMPS) XSTAMPW(12, 7);
                }
                wait_flag(h2ready, tag);
                gh2_dots(br0);
                if (wq < 2) gh2_dots(br1);
                if (!WRNN_XCDS_GRU2_STAMPS) XSTAMPW(13, 5);
            }
        }
        XSTAMP_BAR();
        bar();
        // next step's x, GRU1 terms and the abort word: one LDS round trip
        const int ab = *abort_flag;
        const float xn = xs[t & 1];
        s4 = lds4(sg + 4 * tid);
        s4b = lds4(sg + 4 * u2);
        if (ab) return;
        if (wave != 0) x = xn;
    }
    // ---- carry the recurrent state to the next time chunk (every workgroup its own copy)
    __syncthreads();
    st[tid] = h1v;
    if (two) st[u2] = h1v2;
    for (int i = tid; i < 4 * R; i += kXThreads) st[oSG + i] = sg[i];
    if (tid < 84) st[oGH2 + tid] = gh2s[tid];
    if (wave < kSUB && lane < 4) st[oH2 + ul] = h2own;
    if (tid == 0) st[oX] = xs[(t_end - 1) & 1];
}

#define WRNN_K_XCDS fatchord_xcds_kernel<false>
#define WRNN_K_XCDS_DBG fatchord_xcds_kernel<true>

hipError_t launch_xcds(const XcdsArgs &a, hipStream_t st) {
    XcdsArgs args = a;
    void *params[] = {&args};
    const void *kf = a.dbg ? (const void *)WRNN_K_XCDS_DBG : (const void *)WRNN_K_XCDS;
    return hipLaunchKernel(kf, dim3(kXcds * kXcdWgs), dim3(kXThreads), params, xcds_lds_layout().total * sizeof(float), st);
}

hipError_t prepare_xcds_kernel(int max_lds_bytes) {
    for (const void *kf : {(const void *)WRNN_K_XCDS, (const void *)WRNN_K_XCDS_DBG}) {
        hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds_bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t xcds_occupancy(int *blocks_per_cu) {
    int best = 1 << 30;
    for (const void *kf : {(const void *)WRNN_K_XCDS, (const void *)WRNN_K_XCDS_DBG}) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kf, kXThreads, xcds_lds_layout().total * sizeof(float));
        if (e != hipSuccess) return e;
        best = n < best ? n : best;
    }
    *blocks_per_cu = best;
    return hipSuccess;
}

}  // namespace wrnn
