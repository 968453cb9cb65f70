// capi.cpp — host side of the C-ABI declared in include/wavernn_amd.h.
//
// Owns the device state of one WaveRNN loop: the per-workgroup weight slabs (packed from
// reference state_dict tensors), the I-layer weights for the conditioning GEMM, the
// conditioning-projection workspace, the hand-off granules and the control words.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/wavernn_amd.h"
#include "fatchord_loop.h"
#include "fatchord_rows.h"
#include "deepmind_rows.h"
#include "fatchord_split.h"
#include "fatchord_xcd.h"
#include "fatchord_xcds.h"
#include "fatchord_xcdm.h"
#include "deepmind_xcd.h"

namespace wrnn {
hipError_t launch_ci_gemm(const float *cond, int CD, int Bt, int b0, int Bc, int t0, int L, const float *W, int ldw,
                          const float *bias, int N, int K, float *cI, int ldc, hipStream_t st);
hipError_t launch_pack_cond_input(const float *cond, int CD, int Bt, int b0, int B, int t0, int Lc, int KX, float *X,
                                  hipStream_t st, int split = 0, float one = 1.0f);
hipError_t launch_frame_cond(const float *mel, const float *aux, int U, int feat, int A4, int NF, int frames, int jlo,
                             int kind, float *rec, hipStream_t st);
hipError_t launch_terms_interp(const float *FT, const float *AT, const float *coef, float *T, int N, int U, int NF,
                               int NFF, int hop, int nJ, int nf, int stride, int b0, int nb, int t0, int nt,
                               hipStream_t st);
hipError_t launch_pack_terms_input(const float *cond, int CD, int Bt, int b0, int B, int t0, int Lc, int feat, int A,
                                   int R, int KX, float *X, hipStream_t st);
hipError_t launch_rows(const RowsArgs &a, const RowsGroup *g1, size_t lds_bytes, hipStream_t st);
hipError_t prepare_rows_kernel(int max_lds_bytes);
hipError_t rows_occupancy(int *blocks_per_cu, size_t lds_bytes);
hipError_t launch_dm(const DmArgs &a, const DmGroup *g1, size_t lds_bytes, hipStream_t st);
hipError_t prepare_dm_kernel(int max_lds_bytes);
hipError_t dm_occupancy(int *blocks_per_cu, size_t lds_bytes);
hipError_t launch_loop(const LoopArgs &a, size_t lds_bytes, hipStream_t st);
hipError_t prepare_loop_kernel(int max_lds_bytes);
hipError_t loop_occupancy(int *blocks_per_cu, size_t lds_bytes);
bool loop_has_fast_path(int R, int F, int A, int NC, bool mol, int U, int UF, int UC);
hipError_t launch_split(const SplitArgs &a, size_t lds_bytes, hipStream_t st);
hipError_t prepare_split_kernel(int max_lds_bytes);
hipError_t split_occupancy(int *blocks_per_cu, size_t lds_bytes);
bool split_has_kernel(int R, int F);
hipError_t launch_xcd(const XcdArgs &a, hipStream_t st);
hipError_t prepare_xcd_kernel(int max_lds_bytes);
hipError_t xcd_occupancy(int *blocks_per_cu);
hipError_t launch_xcds(const XcdsArgs &a, hipStream_t st);
hipError_t prepare_xcds_kernel(int max_lds_bytes);
hipError_t xcds_occupancy(int *blocks_per_cu);
hipError_t launch_xcdm(const XcdmArgs &a, int nq, bool raw, hipStream_t st);
hipError_t prepare_xcdm_kernel(int max_lds_bytes);
hipError_t xcdm_max_quads(int max_lds_bytes, bool raw, int *nq_max);
hipError_t launch_philox_fill(float *out, unsigned long long seed, long long row0, int nb, int t0, int Lc, int K, int mol,
                              hipStream_t st);
hipError_t launch_dx(const DxArgs &a, hipStream_t st);
hipError_t prepare_dx_kernel(int max_lds_bytes, bool *ok);
int cond_fail(int code, const std::string &m);
}  // namespace wrnn

using namespace wrnn;

// One partition of the loop weights over the multi-row kernel's workgroups (see wrnn_ctx).
struct RowsPart {
    RowsSlab rs{};
    int rU = 0, rG = 0, rUF = 0, rUC = 0, NT = 0;
    bool ok = false;
    float *d_slab = nullptr, *d_Wt = nullptr;
};

// The deepmind partition (units per workgroup, grid) and its packed slab (see wrnn_ctx::dm2)
struct DmPart {
    DmSlab ds{};
    int dmU = 0, dmUO = 0, dmUO2 = 0, G = 0;
    bool ok = false;
    float *d_slab = nullptr;
};

struct wrnn_ctx {
    wrnn_config cfg{};
    int device = 0;
    int num_cus = 0;
    int max_lds = 0;
    int G = 0, U = 0, UF = 0, UC = 0, NMAX = 0, NK = 0, CD = 0;
    int max_rows = 0;
    SlabLayout s{};
    std::map<std::string, std::vector<float>> w;   // loop tensors, host copies
    bool ready = false;
    float *d_slab = nullptr, *d_IW = nullptr, *d_Ib = nullptr;
    float *d_cI = nullptr;
    size_t cI_cap = 0;                              // floats
    unsigned long long *d_xg = nullptr;
    size_t xg_cap = 0;                              // granules
    int *d_ctl = nullptr;
    long long timeout_ticks = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    std::string err;
    // multi-row (fold-batched) path: fatchord_rows.hip
    RowsSlab rs{};
    int rU = 0, rG = 0, rUF = 0, rUC = 0;           // rows-kernel partition (U = 4 when sparse)
    bool sparse = false;                            // GRU weights stored as nonzero 4x4 blocks
    int NT = 0, KX = 0, KA = 0;
    int KXc = 0;                                    // XCD kernels' terms-GEMM depth: [cond record | 1 0 0 0]
    bool rows_ok = false;                           // weights fit LDS with at least one row (or stream)
    bool rows_gw = false;                           // dense weights exceed LDS: the slab is streamed from HBM
    float *d_rslab = nullptr, *d_Wt = nullptr;      // per-workgroup slabs, terms-GEMM weights [G·NT][KX]
    float *d_X = nullptr, *d_T = nullptr, *d_act = nullptr, *d_state = nullptr;
    size_t X_cap = 0, T_cap = 0, act_cap = 0, state_cap = 0;   // floats
    unsigned *d_flags = nullptr;                    // [2 row groups][kRowsHops][kFlagSlots][kFlagStride]
    unsigned long long *d_xr = nullptr;             // x granules, [2 row groups][kXReps][kXRepStride]
    unsigned long long *d_gact = nullptr;           // rows granule mode: [2 row groups][kRowsHops][gstride]
    size_t gact_cap = 0;
    // the same weights over G/2 workgroups (twice the units each) for two row groups per launch
    // (large B: halves the activation rows every workgroup streams per stage); swapped into the
    // r* fields above while in use
    RowsPart g2{};
    rocblas_handle blas = nullptr;
    int last_path = 0;                              // 1 = latency, 2 = rows, 3 = deepmind, 4 = split, 5 = xcd, 6 = xcd sparse
    // deepmind_version (WRNN_MODE_DM): deepmind_rows.hip
    DmSlab ds{};
    int dmU = 0, dmUO = 0, dmUO2 = 0;
    bool dm = false;
    bool dm_gw = false;                             // the DM slab exceeds LDS: streamed from HBM
    float *d_dmslab = nullptr;
    DmPart dm2{};                                   // G/2 workgroups, twice the units: two row groups per launch
    unsigned *d_dmflags = nullptr;
    unsigned long long *d_dmxg = nullptr;
    size_t dmflags_cap = 0, dmxg_cap = 0;
    // batch-1 MoL role-split kernel: fatchord_split.hip
    bool split_ok = false;
    int sGg = 0, sGf = 0;
    SplitGruSlab sgs{};
    SplitFcSlab sfs{};
    float *d_sgslab = nullptr, *d_sfslab = nullptr, *d_sWt = nullptr;
    // XCD-resident MoL kernel (rnn / fc 512): fatchord_xcd.hip
    bool xcd_ok = false;
    XcdSlab xs{};
    float *d_xslab = nullptr, *d_xWt = nullptr, *d_xstate = nullptr;
    size_t xstate_cap = 0;
    unsigned long long *d_xgx = nullptr;
    int *d_members = nullptr;
    // XCD-resident MoL kernel for rnn 896 with 4x4 block-sparse GRU weights: fatchord_xcds.hip
    // (shares the d_x* buffers: the dense one needs rnn 512); cap = dims and device fit, ok =
    // the loaded weights are block-sparse with <= kSNB nonzero blocks per gate block-row
    bool xcds_cap = false, xcds_ok = false;
    XcdsSlab xss{};
    // XCD-resident many-row MoL kernel (rnn / fc 512, MFMA): fatchord_xcdm.hip; shares the XCD
    // kernel's terms-GEMM weights (d_xWt)
    bool xcdm_ok = false;
    int xcdm_nq = 0;                                // largest co-resident quad count (rows per XCD / 4)
    XcdmSlab xms{};
    float *d_xmslab = nullptr, *d_xmstate = nullptr, *d_xmnoise = nullptr;
    float *d_xmWt = nullptr;   // many-row kernel's terms-GEMM weights: the first kMRing rows of each workgroup's record
    size_t xmnoise_cap = 0;
    // XCD-resident deepmind kernel (hidden 896, quantisation 256, MFMA): deepmind_xcd.hip
    bool dx_ok = false;
    float *d_dxslab = nullptr, *d_dxstate = nullptr, *d_dxnoise = nullptr;
    size_t dxnoise_cap = 0;
    unsigned long long *d_dxxg = nullptr;
    unsigned long long *d_xmxg = nullptr;
    // frame-rate conditioning terms (wrnn_generate_frames, frame_terms.hip): the cascade's
    // per-phase frame weights, W·(mel frame) and W·(aux frame, ones) rows, their GEMM input
    // records, and the per-sample conditioning of the paths that still take it
    float *d_coef = nullptr, *d_FT = nullptr, *d_AT = nullptr, *d_frec = nullptr, *d_cond = nullptr;
    size_t coef_cap = 0, FT_cap = 0, AT_cap = 0, frec_cap = 0, cond_cap = 0;
    std::vector<float> coef_host;                   // the table d_coef holds (re-uploaded when it changes)
};

namespace {

const int kCtlWords = 8;

int fail(wrnn_t *h, int code, const std::string &msg) {
    if (h) h->err = msg;
    return code;
}

#define HIP_TRY(h, expr)                                                                      \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            return fail((h), WRNN_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));   \
    } while (0)

struct Need {
    const char *name;
    int64_t rows, cols;
};

std::vector<Need> required(const wrnn_config &c) {
    if (c.mode == WRNN_MODE_DM) {   // deepmind_version.py:14-31
        const int64_t H = c.rnn_dims, S = H / 2, Q = c.n_classes;
        return {{"R.weight", 3 * H, H},      {"O1.weight", S, S},        {"O1.bias", S, 1},
                {"O2.weight", Q, S},         {"O2.bias", Q, 1},          {"O3.weight", S, S},
                {"O3.bias", S, 1},           {"O4.weight", Q, S},        {"O4.bias", Q, 1},
                {"I_coarse.weight", 3 * S, 2}, {"I_fine.weight", 3 * S, 3}, {"bias_u", H, 1},
                {"bias_r", H, 1},            {"bias_e", H, 1}};
    }
    const int64_t R = c.rnn_dims, F = c.fc_dims, A = c.aux_dims, M = c.feat_dims, NC = c.n_classes;
    return {{"I.weight", R, 1 + M + A},      {"I.bias", R, 1},
            {"rnn1.weight_ih_l0", 3 * R, R}, {"rnn1.weight_hh_l0", 3 * R, R},
            {"rnn1.bias_ih_l0", 3 * R, 1},   {"rnn1.bias_hh_l0", 3 * R, 1},
            {"rnn2.weight_ih_l0", 3 * R, R + A}, {"rnn2.weight_hh_l0", 3 * R, R},
            {"rnn2.bias_ih_l0", 3 * R, 1},   {"rnn2.bias_hh_l0", 3 * R, 1},
            {"fc1.weight", F, R + A},        {"fc1.bias", F, 1},
            {"fc2.weight", F, F + A},        {"fc2.bias", F, 1},
            {"fc3.weight", NC, F},           {"fc3.bias", NC, 1}};
}

SlabLayout make_slab_layout(const wrnn_ctx &h) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, A = h.cfg.aux_dims, NC = h.cfg.n_classes;
    const bool mol = h.cfg.mode == WRNN_MODE_MOL;
    SlabLayout s{};
    int o = 0;
    auto take = [&](int n) { int at = o; o += round4(n); return at; };
    s.wih1 = take(3 * h.U * R);
    s.whh1 = take(3 * h.U * R);
    s.wih2 = take(3 * h.U * (R + A));
    s.whh2 = take(3 * h.U * R);
    s.bih1 = take(3 * h.U);
    s.bhh1 = take(3 * h.U);
    s.bih2 = take(3 * h.U);
    s.bhh2 = take(3 * h.U);
    s.w1 = take(h.UF * (R + A));
    s.b1 = take(h.UF);
    s.w2 = take(h.UF * (F + A));
    s.b2 = take(h.UF);
    s.w3 = take((mol ? NC : h.UC) * F);
    s.b3 = take(mol ? NC : h.UC);
    s.wi0 = take(R);
    s.total = o;
    return s;
}

// Pack workgroup w's rows: GRU gate rows (g·R + j) for owned units j, fc rows, fc3 rows.
void pack_slab(const wrnn_ctx &h, int w, float *out) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, A = h.cfg.aux_dims, NC = h.cfg.n_classes;
    const bool mol = h.cfg.mode == WRNN_MODE_MOL;
    const SlabLayout &s = h.s;
    std::fill(out, out + s.total, 0.0f);
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    for (int u = 0; u < h.U; ++u) {
        const int j = w * h.U + u;
        if (j >= R) continue;
        for (int g = 0; g < 3; ++g) {
            const int src = g * R + j, dst = g * h.U + u;
            std::memcpy(out + s.wih1 + (size_t)dst * R, W("rnn1.weight_ih_l0") + (size_t)src * R, R * 4);
            std::memcpy(out + s.whh1 + (size_t)dst * R, W("rnn1.weight_hh_l0") + (size_t)src * R, R * 4);
            std::memcpy(out + s.wih2 + (size_t)dst * (R + A), W("rnn2.weight_ih_l0") + (size_t)src * (R + A),
                        (R + A) * 4);
            std::memcpy(out + s.whh2 + (size_t)dst * R, W("rnn2.weight_hh_l0") + (size_t)src * R, R * 4);
            out[s.bih1 + dst] = W("rnn1.bias_ih_l0")[src];
            out[s.bhh1 + dst] = W("rnn1.bias_hh_l0")[src];
            out[s.bih2 + dst] = W("rnn2.bias_ih_l0")[src];
            out[s.bhh2 + dst] = W("rnn2.bias_hh_l0")[src];
        }
    }
    for (int r = 0; r < h.UF; ++r) {
        const int j = w * h.UF + r;
        if (j >= F) continue;
        std::memcpy(out + s.w1 + (size_t)r * (R + A), W("fc1.weight") + (size_t)j * (R + A), (R + A) * 4);
        std::memcpy(out + s.w2 + (size_t)r * (F + A), W("fc2.weight") + (size_t)j * (F + A), (F + A) * 4);
        out[s.b1 + r] = W("fc1.bias")[j];
        out[s.b2 + r] = W("fc2.bias")[j];
    }
    if (mol) {
        std::memcpy(out + s.w3, W("fc3.weight"), (size_t)NC * F * 4);
        std::memcpy(out + s.b3, W("fc3.bias"), (size_t)NC * 4);
    } else {
        for (int r = 0; r < h.UC; ++r) {
            const int j = w * h.UC + r;
            if (j >= NC) continue;
            std::memcpy(out + s.w3 + (size_t)r * F, W("fc3.weight") + (size_t)j * F, F * 4);
            out[s.b3 + r] = W("fc3.bias")[j];
        }
    }
    const float *IW = W("I.weight");
    const int nin = 1 + h.cfg.feat_dims + A;
    for (int j = 0; j < R; ++j) out[s.wi0 + j] = IW[(size_t)j * nin];
}

RowsSlab make_rows_slab(const wrnn_ctx &h, int nbmax) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, NC = h.cfg.n_classes;
    const bool mol = h.cfg.mode == WRNN_MODE_MOL;
    const int dense = nbmax > 0 ? 0 : 1;
    RowsSlab s{};
    int o = 0;
    auto take = [&](int n) { int at = o; o += round4(n); return at; };
    s.wih2 = take(dense * 3 * h.rU * R);
    s.whh1 = take(dense * 3 * h.rU * R);
    s.whh2 = take(dense * 3 * h.rU * R);
    s.sp = take(9 * nbmax * 16);
    s.spc = take(9 * nbmax);
    s.spn = take(nbmax > 0 ? 9 : 0);
    s.nbmax = nbmax;
    s.w1 = take(h.rUF * R);
    s.w2 = take(h.rUF * F);
    if (!mol) {
        s.w3 = take(h.rUC * F);
        s.b3 = take(h.rUC);
    }
    s.bih1 = take(3 * h.rU);
    s.bhh1 = take(3 * h.rU);
    s.bih2 = take(3 * h.rU);
    s.bhh2 = take(3 * h.rU);
    s.q1 = take(3 * h.rU);
    s.q2 = take(3 * h.rU);
    s.q3 = take(h.rUF);
    s.body = o;          // everything before the MoL head: always LDS-resident
    if (mol) {           // the replicated 30-row head last, so a launch may leave it in HBM
        s.w3 = take(NC * F);
        s.b3 = take(NC);
    }
    s.total = o;
    return s;
}

// The three GRU matrices the rows kernel multiplies in the loop, as (tensor, row stride):
// W_ih2[:, :R] (stride R + A), W_hh1, W_hh2 (SparseMat order).
struct LoopMat {
    const float *w;
    int ld;
};
void loop_mats(const wrnn_ctx &h, LoopMat (&m)[3]) {
    const int R = h.cfg.rnn_dims, A = h.cfg.aux_dims;
    m[SP_WIH2] = {h.w.at("rnn2.weight_ih_l0").data(), R + A};
    m[SP_WHH1] = {h.w.at("rnn1.weight_hh_l0").data(), R};
    m[SP_WHH2] = {h.w.at("rnn2.weight_hh_l0").data(), R};
}

bool block_nonzero(const float *w, int ld, int r0, int c0) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            if (w[(size_t)(r0 + r) * ld + c0 + c] != 0.0f) return true;
    return false;
}

// Largest nonzero-block count of any gate block-row (4 rows) of the three loop matrices, and the
// overall block density; the rows kernel goes sparse when density <= 1/2.
void block_stats(const wrnn_ctx &h, int *nbmax, double *density) {
    const int R = h.cfg.rnn_dims;
    LoopMat m[3];
    loop_mats(h, m);
    long long nz = 0, tot = 0;
    int mx = 0;
    for (int k = 0; k < 3; ++k)
        for (int rb = 0; rb < 3 * R; rb += 4) {
            int n = 0;
            for (int cb = 0; cb < R; cb += 4) n += block_nonzero(m[k].w, m[k].ld, rb, cb);
            nz += n;
            tot += R / 4;
            mx = std::max(mx, n);
        }
    *nbmax = mx;
    *density = tot ? (double)nz / tot : 1.0;
}

// x-column constants Q = W[:, :R]·W_I[:, 0] (fp32, sequential)
float xcol_dot(const float *wrow, const float *IW, int nin, int R) {
    float acc = 0.0f;
    for (int k = 0; k < R; ++k) acc = std::fma(wrow[k], IW[(size_t)k * nin], acc);
    return acc;
}

void pack_rows_slab(const wrnn_ctx &h, int w, float *out) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, A = h.cfg.aux_dims, NC = h.cfg.n_classes;
    const bool mol = h.cfg.mode == WRNN_MODE_MOL;
    const RowsSlab &s = h.rs;
    const int U = h.rU, UF = h.rUF, UC = h.rUC;
    std::fill(out, out + s.total, 0.0f);
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    const float *IW = W("I.weight");
    const int nin = 1 + h.cfg.feat_dims + A;
    for (int u = 0; u < U; ++u) {
        const int j = w * U + u;
        if (j >= R) continue;
        for (int g = 0; g < 3; ++g) {
            const int src = g * R + j, dst = g * U + u;
            const float *ih1 = W("rnn1.weight_ih_l0") + (size_t)src * R;
            const float *ih2 = W("rnn2.weight_ih_l0") + (size_t)src * (R + A);
            if (s.nbmax == 0) {
                std::memcpy(out + s.wih2 + (size_t)dst * R, ih2, R * 4);
                std::memcpy(out + s.whh1 + (size_t)dst * R, W("rnn1.weight_hh_l0") + (size_t)src * R, R * 4);
                std::memcpy(out + s.whh2 + (size_t)dst * R, W("rnn2.weight_hh_l0") + (size_t)src * R, R * 4);
            }
            out[s.bih1 + dst] = W("rnn1.bias_ih_l0")[src];
            out[s.bhh1 + dst] = W("rnn1.bias_hh_l0")[src];
            out[s.bih2 + dst] = W("rnn2.bias_ih_l0")[src];
            out[s.bhh2 + dst] = W("rnn2.bias_hh_l0")[src];
            out[s.q1 + dst] = xcol_dot(ih1, IW, nin, R);
            out[s.q2 + dst] = xcol_dot(ih2, IW, nin, R);
        }
    }
    if (s.nbmax > 0) {   // this workgroup's block-row (units 4w..4w+3) of each gate, nonzero blocks only
        LoopMat m[3];
        loop_mats(h, m);
        int *col = reinterpret_cast<int *>(out + s.spc);
        int *cnt = reinterpret_cast<int *>(out + s.spn);
        for (int k = 0; k < 3; ++k)
            for (int g = 0; g < 3; ++g) {
                const int r0 = g * R + 4 * w, sl = k * 3 + g;
                int n = 0;
                for (int cb = 0; cb < R; cb += 4) {
                    if (!block_nonzero(m[k].w, m[k].ld, r0, cb)) continue;
                    float *blk = out + s.sp + ((size_t)sl * s.nbmax + n) * 16;
                    for (int r = 0; r < 4; ++r)
                        for (int c = 0; c < 4; ++c) blk[r * 4 + c] = m[k].w[(size_t)(r0 + r) * m[k].ld + cb + c];
                    col[sl * s.nbmax + n] = cb / 4;
                    ++n;
                }
                cnt[sl] = n;
            }
    }
    for (int r = 0; r < UF; ++r) {
        const int j = w * UF + r;
        if (j >= F) continue;
        const float *w1 = W("fc1.weight") + (size_t)j * (R + A);
        std::memcpy(out + s.w1 + (size_t)r * R, w1, R * 4);
        std::memcpy(out + s.w2 + (size_t)r * F, W("fc2.weight") + (size_t)j * (F + A), F * 4);
        out[s.q3 + r] = xcol_dot(w1, IW, nin, R);
    }
    if (mol) {
        std::memcpy(out + s.w3, W("fc3.weight"), (size_t)NC * F * 4);
        std::memcpy(out + s.b3, W("fc3.bias"), (size_t)NC * 4);
    } else {
        for (int r = 0; r < UC; ++r) {
            const int j = w * UC + r;
            if (j >= NC) continue;
            std::memcpy(out + s.w3 + (size_t)r * F, W("fc3.weight") + (size_t)j * F, F * 4);
            out[s.b3 + r] = W("fc3.bias")[j];
        }
    }
}

// Weights of the conditioning-terms GEMM: row w·NT + k of [G·NT][KX] against X = [cI | a2 a3 a4 | 1 0 0 0]
void pack_terms_weights(const wrnn_ctx &h, float *Wt) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, A = h.cfg.aux_dims, U = h.rU, UF = h.rUF, KX = h.KX;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    std::fill(Wt, Wt + (size_t)h.rG * h.NT * KX, 0.0f);
    for (int w = 0; w < h.rG; ++w)
        for (int k = 0; k < 6 * U + 2 * UF; ++k) {
            float *row = Wt + ((size_t)w * h.NT + k) * KX;
            if (k < 6 * U) {
                const int kk = k % (3 * U), g = kk / U, j = w * U + kk % U;
                if (j >= R) continue;
                if (k < 3 * U) {
                    std::memcpy(row, W("rnn1.weight_ih_l0") + (size_t)(g * R + j) * R, R * 4);
                } else {
                    const float *ih2 = W("rnn2.weight_ih_l0") + (size_t)(g * R + j) * (R + A);
                    std::memcpy(row, ih2, R * 4);
                    std::memcpy(row + R, ih2 + R, A * 4);                       // a2
                }
            } else if (k < 6 * U + UF) {
                const int r = w * UF + (k - 6 * U);
                if (r >= F) continue;
                const float *w1 = W("fc1.weight") + (size_t)r * (R + A);
                std::memcpy(row, w1, R * 4);
                std::memcpy(row + R + A, w1 + R, A * 4);                        // a3
                row[R + 3 * A] = W("fc1.bias")[r];
            } else {
                const int r = w * UF + (k - 6 * U - UF);
                if (r >= F) continue;
                std::memcpy(row + R + 2 * A, W("fc2.weight") + (size_t)r * (F + A) + F, A * 4);   // a4
                row[R + 3 * A] = W("fc2.bias")[r];
            }
        }
}

void fold_ci_row(const wrnn_ctx &h, const float *w, float *dst);

// MoL: the same slots against the composed input X' = [mel | a1 | a2 | a3 | a4 | 1 0 0 0]
// (KXc = CD + 4) — the I layer folded into the W_ih1 / W_ih2 / fc1 rows in fp64 (fold_ci_row,
// as the XCD kernels' terms), so the GEMM needs no cI and runs at depth 212 instead of R + 3A + 4
// (2.9x less work at rnn 512).  RAW keeps the cI GEMM (its labels are checked bit-exact).
bool rows_terms_composed(const wrnn_ctx &h) { return h.cfg.mode == WRNN_MODE_MOL; }
int rows_terms_kx(const wrnn_ctx &h) { return rows_terms_composed(h) ? h.KXc : h.KX; }

void pack_terms_weights_composed(const wrnn_ctx &h, float *Wt) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, M = h.cfg.feat_dims, A = h.cfg.aux_dims, U = h.rU, UF = h.rUF;
    const int KX = h.KXc;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    std::fill(Wt, Wt + (size_t)h.rG * h.NT * KX, 0.0f);
    for (int w = 0; w < h.rG; ++w)
        for (int k = 0; k < 6 * U + 2 * UF; ++k) {
            float *row = Wt + ((size_t)w * h.NT + k) * KX;
            if (k < 6 * U) {
                const int kk = k % (3 * U), g = kk / U, j = w * U + kk % U;
                if (j >= R) continue;
                if (k < 3 * U) {
                    fold_ci_row(h, W("rnn1.weight_ih_l0") + (size_t)(g * R + j) * R, row);
                } else {
                    const float *ih2 = W("rnn2.weight_ih_l0") + (size_t)(g * R + j) * (R + A);
                    fold_ci_row(h, ih2, row);
                    for (int a = 0; a < A; ++a) row[M + A + a] += ih2[R + a];                   // a2
                }
            } else if (k < 6 * U + UF) {
                const int r = w * UF + (k - 6 * U);
                if (r >= F) continue;
                const float *w1 = W("fc1.weight") + (size_t)r * (R + A);
                fold_ci_row(h, w1, row);
                for (int a = 0; a < A; ++a) row[M + 2 * A + a] += w1[R + a];                    // a3
                row[h.CD] += W("fc1.bias")[r];
            } else {
                const int r = w * UF + (k - 6 * U - UF);
                if (r >= F) continue;
                for (int a = 0; a < A; ++a) row[M + 3 * A + a] = W("fc2.weight")[(size_t)r * (F + A) + F + a];   // a4
                row[h.CD] = W("fc2.bias")[r];
            }
        }
}

size_t rows_lds_bytes(const wrnn_ctx &h, int B, int TB, bool head_lds = true) {
    const int slab = h.rows_gw ? 0 : head_lds ? h.rs.total : h.rs.body;
    return (size_t)rows_lds_layout(slab, B, TB, h.cfg.rnn_dims, h.cfg.fc_dims,
                                   h.cfg.n_classes, h.NK, h.rU, h.rUF, h.rG)
               .total * sizeof(float);
}

// (Re)derive the rows-kernel partition: dense = the latency kernel's; sparse = one 4-unit
// block-row per workgroup (G = R / 4).  Sets rows_ok.
int rows_tile_for(const wrnn_ctx &h, int B, bool head_lds = true);
void set_rows_partition(wrnn_ctx &h, int nbmax) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims;
    const bool mol = h.cfg.mode == WRNN_MODE_MOL;
    h.sparse = nbmax > 0;
    if (h.sparse) {
        h.rU = 4;
        h.rG = R / 4;
    } else {
        h.rU = h.U;
        h.rG = h.G;
    }
    h.rUF = (F + h.rG - 1) / h.rG;
    h.rUC = mol ? 0 : (h.cfg.n_classes + h.rG - 1) / h.rG;
    h.NT = rows_terms(h.rU, h.rUF);
    h.rs = make_rows_slab(h, nbmax);
    h.rows_gw = false;
    h.rows_ok = rows_tile_for(h, 1) > 0;
    // dense weights beyond the grid's LDS: the same kernel with the slab streamed from HBM
    if (!h.rows_ok && nbmax == 0) {
        h.rows_gw = true;
        h.rows_ok = rows_tile_for(h, 1) > 0;
    }
}

// Largest tile (<= 16 rows; up to 32 with the MoL head left in HBM) that fits next to B rows of
// state; 0 if none does
int rows_tile_for(const wrnn_ctx &h, int B, bool head_lds) {
    for (int tb = std::min(B, head_lds ? 16 : 32); tb >= 1; --tb)
        if (rows_lds_bytes(h, B, tb, head_lds) <= (size_t)h.max_lds) return tb;
    return 0;
}

void swap_part(wrnn_ctx &h, RowsPart &p) {
    std::swap(h.rs, p.rs);
    std::swap(h.rU, p.rU);
    std::swap(h.rG, p.rG);
    std::swap(h.rUF, p.rUF);
    std::swap(h.rUC, p.rUC);
    std::swap(h.NT, p.NT);
    std::swap(h.rows_ok, p.ok);
    std::swap(h.d_rslab, p.d_slab);
    std::swap(h.d_Wt, p.d_Wt);
}

// Swaps a partition in for a scope
struct PartScope {
    wrnn_ctx &h;
    RowsPart &p;
    bool on;
    PartScope(wrnn_ctx &h_, RowsPart &p_, bool on_) : h(h_), p(p_), on(on_) {
        if (on) swap_part(h, p);
    }
    ~PartScope() {
        if (on) swap_part(h, p);
    }
};

// The two-group partition: dense weights over G/2 workgroups (G even)
void set_group_partition(wrnn_ctx &h) {
    h.g2 = RowsPart{};
    if (h.G % 2 || h.G < 8 || h.rows_gw) return;
    RowsPart flat{};
    swap_part(h, flat);   // h.r* empty, flat holds the current partition
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims;
    const bool mol = h.cfg.mode == WRNN_MODE_MOL;
    h.rG = h.G / 2;
    h.rU = (R + h.rG - 1) / h.rG;
    h.rUF = (F + h.rG - 1) / h.rG;
    h.rUC = mol ? 0 : (h.cfg.n_classes + h.rG - 1) / h.rG;
    h.NT = rows_terms(h.rU, h.rUF);
    h.rs = make_rows_slab(h, 0);
    h.rows_ok = rows_tile_for(h, 16, false) >= 4;
    swap_part(h, flat);   // h.r* = flat again, `flat` = the group partition
    h.g2 = flat;
}

// ------------------------------------------------------------------ deepmind_version packing
DmSlab make_dm_slab(const wrnn_ctx &h) {
    const int H = h.cfg.rnn_dims, S = H / 2;
    DmSlab s{};
    int o = 0;
    auto take = [&](int n) { int at = o; o += round4(n); return at; };
    s.rw = take(6 * h.dmU * H);
    s.o1 = take(h.dmUO * S);
    s.o1b = take(h.dmUO);
    s.o3 = take(h.dmUO * S);
    s.o3b = take(h.dmUO);
    s.o2 = take(h.dmUO2 * S);
    s.o2b = take(h.dmUO2);
    s.o4 = take(h.dmUO2 * S);
    s.o4b = take(h.dmUO2);
    s.ic = take(3 * h.dmU * 2);
    s.if_ = take(3 * h.dmU * 3);
    s.bu = take(2 * h.dmU);
    s.br = take(2 * h.dmU);
    s.be = take(2 * h.dmU);
    s.total = o;
    return s;
}

// Workgroup w: coarse units j = w·U + u and fine units S + j; R rows g·H + half·S + j (g = u, r, e,
// the split of deepmind_version.py:116-119); output rows w·UO + r of O1/O3, w·UO2 + r of O2/O4.
void pack_dm_slab(const wrnn_ctx &h, int w, float *out) {
    const int H = h.cfg.rnn_dims, S = H / 2, Q = h.cfg.n_classes, U = h.dmU;
    const DmSlab &s = h.ds;
    std::fill(out, out + s.total, 0.0f);
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    for (int u = 0; u < U; ++u) {
        const int j = w * U + u;
        if (j >= S) continue;
        for (int half = 0; half < 2; ++half)
            for (int g = 0; g < 3; ++g) {
                std::memcpy(out + s.rw + (size_t)((half * 3 + g) * U + u) * H,
                            W("R.weight") + (size_t)(g * H + half * S + j) * H, H * 4);
                const float *bias = W(g == 0 ? "bias_u" : g == 1 ? "bias_r" : "bias_e");
                out[(g == 0 ? s.bu : g == 1 ? s.br : s.be) + half * U + u] = bias[half * S + j];
            }
        for (int g = 0; g < 3; ++g) {
            for (int k = 0; k < 2; ++k) out[s.ic + (g * U + u) * 2 + k] = W("I_coarse.weight")[(g * S + j) * 2 + k];
            for (int k = 0; k < 3; ++k) out[s.if_ + (g * U + u) * 3 + k] = W("I_fine.weight")[(g * S + j) * 3 + k];
        }
    }
    for (int r = 0; r < h.dmUO; ++r) {
        const int j = w * h.dmUO + r;
        if (j >= S) continue;
        std::memcpy(out + s.o1 + (size_t)r * S, W("O1.weight") + (size_t)j * S, S * 4);
        std::memcpy(out + s.o3 + (size_t)r * S, W("O3.weight") + (size_t)j * S, S * 4);
        out[s.o1b + r] = W("O1.bias")[j];
        out[s.o3b + r] = W("O3.bias")[j];
    }
    for (int r = 0; r < h.dmUO2; ++r) {
        const int j = w * h.dmUO2 + r;
        if (j >= Q) continue;
        std::memcpy(out + s.o2 + (size_t)r * S, W("O2.weight") + (size_t)j * S, S * 4);
        std::memcpy(out + s.o4 + (size_t)r * S, W("O4.weight") + (size_t)j * S, S * 4);
        out[s.o2b + r] = W("O2.bias")[j];
        out[s.o4b + r] = W("O4.bias")[j];
    }
}

// ---- XCD-resident deepmind kernel (deepmind_xcd.h): the slab of workgroup c (the same on every
// XCD, replicated 8×): A operands [wave][DxA][lane] and constants
void pack_dx_slab(const wrnn_ctx &h, std::vector<float> &slab) {
    const int H = kDxH, S = kDxS, U = kDxU;
    const DxSlab L = dx_slab_layout();
    slab.assign((size_t)kXcds * kXcdWgs * L.total, 0.0f);
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    const float *R = W("R.weight"), *O1 = W("O1.weight"), *O3 = W("O3.weight"), *O2 = W("O2.weight"), *O4 = W("O4.weight");
    std::vector<float> one((size_t)L.total);
    for (int c = 0; c < kXcdWgs; ++c) {
        std::fill(one.begin(), one.end(), 0.0f);
        // WG-local R row rr = (half·3 + g)·14 + u → R row g·H + half·S + 14c + u
        auto rrow = [&](int rr) {
            const int half = rr / (3 * U), g = (rr / U) % 3, u = rr % U;
            return R + (size_t)(g * H + half * S + U * c + u) * H;
        };
        for (int w = 0; w < kDxWaves; ++w)
            for (int l = 0; l < 64; ++l) {
                const int j = l & 3, b = l >> 2, g4 = b & 3, sp = b >> 2, g2 = b & 1, ks = b >> 1;
                float *A = one.data() + L.a + (size_t)w * kDxA * 64 + l;
                for (int s = 0; s < 5; ++s) {
                    const float *row = rrow(16 * s + 4 * g4 + j);
                    for (int m = 0; m < 56; ++m) {
                        const int col = (m < 28 ? 0 : S) + kDxKW * w + 28 * sp + (m % 28);
                        A[(DA_R + 56 * s + m) * 64] = row[col];
                    }
                }
                {
                    const float *row = rrow(80 + j);
                    for (int m = 0; m < 14; ++m) A[(DA_RQ + m) * 64] = row[(m < 7 ? 0 : S) + kDxKW * w + 7 * b + (m % 7)];
                }
                const int r13 = 4 * g4 + j;
                if (r13 < U)
                    for (int m = 0; m < 28; ++m) {
                        const int col = kDxKW * w + 28 * sp + m;
                        A[(DA_O1 + m) * 64] = O1[(size_t)(U * c + r13) * S + col];
                        A[(DA_O3 + m) * 64] = O3[(size_t)(U * c + r13) * S + col];
                    }
                const int r24 = 4 * g2 + j;
                for (int m = 0; m < 14; ++m) {
                    const int col = kDxKW * w + 14 * ks + m;
                    A[(DA_O2 + m) * 64] = O2[(size_t)(kDxUO2 * c + r24) * S + col];
                    A[(DA_O4 + m) * 64] = O4[(size_t)(kDxUO2 * c + r24) * S + col];
                }
            }
        float *C = one.data() + L.cst;
        for (int r = 0; r < U; ++r) {
            C[DC_B1 + r] = W("O1.bias")[U * c + r];
            C[DC_B3 + r] = W("O3.bias")[U * c + r];
        }
        for (int r = 0; r < kDxUO2; ++r) {
            C[DC_B2 + r] = W("O2.bias")[kDxUO2 * c + r];
            C[DC_B4 + r] = W("O4.bias")[kDxUO2 * c + r];
        }
        for (int g = 0; g < 3; ++g)
            for (int u = 0; u < U; ++u) {
                const int j = U * c + u;
                for (int q = 0; q < 2; ++q) C[DC_IC + (g * U + u) * 2 + q] = W("I_coarse.weight")[(g * S + j) * 2 + q];
                for (int q = 0; q < 3; ++q) C[DC_IF + (g * U + u) * 3 + q] = W("I_fine.weight")[(g * S + j) * 3 + q];
            }
        for (int half = 0; half < 2; ++half)
            for (int u = 0; u < U; ++u) {
                C[DC_BU + half * U + u] = W("bias_u")[half * S + U * c + u];
                C[DC_BR + half * U + u] = W("bias_r")[half * S + U * c + u];
                C[DC_BE + half * U + u] = W("bias_e")[half * S + U * c + u];
            }
        for (int k = 0; k < kXcds; ++k)
            std::copy(one.begin(), one.end(), slab.begin() + (size_t)(k * kXcdWgs + c) * L.total);
    }
}

size_t dm_lds_bytes(const wrnn_ctx &h, int B, int TB) {
    const int S = h.cfg.rnn_dims / 2;
    return (size_t)dm_lds_layout(h.dm_gw ? 0 : h.ds.total, B, TB, S, h.cfg.n_classes, h.dmU, h.G).total * sizeof(float);
}

int dm_tile_for(const wrnn_ctx &h, int B) {
    for (int tb = std::min(B, 16); tb >= 1; --tb)
        if (dm_lds_bytes(h, B, tb) <= (size_t)h.max_lds) return tb;
    return 0;
}

void swap_dm(wrnn_ctx &h, DmPart &p) {
    std::swap(h.ds, p.ds);
    std::swap(h.dmU, p.dmU);
    std::swap(h.dmUO, p.dmUO);
    std::swap(h.dmUO2, p.dmUO2);
    std::swap(h.G, p.G);
    std::swap(h.d_dmslab, p.d_slab);
}

struct DmScope {
    wrnn_ctx &h;
    DmPart &p;
    bool on;
    DmScope(wrnn_ctx &h_, DmPart &p_, bool on_) : h(h_), p(p_), on(on_) {
        if (on) swap_dm(h, p);
    }
    ~DmScope() {
        if (on) swap_dm(h, p);
    }
};

size_t lds_bytes_for(const wrnn_ctx &h, int Bc) {
    return (size_t)lds_layout(h.s.total, Bc, h.cfg.rnn_dims, h.cfg.fc_dims, h.cfg.aux_dims, h.cfg.n_classes, h.NK,
                              h.U, h.UF)
               .total * sizeof(float);
}

// ------------------------------------------------------------- batch-1 role-split kernel
// GRU workgroup g owns units 4g..4g+3 (rows u·3 + gate), FC workgroup f owns fc rows 16f..16f+15
// and the fc3 columns of those rows (fatchord_split.h, slabs).
void make_split_slabs(wrnn_ctx &h) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, NC = h.cfg.n_classes;
    constexpr int U = kSplitUnits, NF = kSplitFcRows;
    int o = 0;
    auto take = [&](int n) { int at = o; o += round4(n); return at; };
    SplitGruSlab &g = h.sgs;
    g.b3 = take(NC);
    g.wih2 = take(3 * U * R);
    g.whh1 = take(3 * U * R);
    g.whh2 = take(3 * U * R);
    g.q1a = take(3 * R);
    g.q2 = take(3 * U);
    g.wi0 = take(U);
    g.bih1 = take(3 * U);
    g.bhh1 = take(3 * U);
    g.bih2 = take(3 * U);
    g.bhh2 = take(3 * U);
    g.total = o;
    o = 0;
    SplitFcSlab &f = h.sfs;
    f.w3p = take(NF * kSplitLogitLine);
    f.w1 = take(NF * R);
    f.w2 = take(NF * F);
    f.total = o;
}

size_t split_lds_bytes(const wrnn_ctx &h) {
    return (size_t)split_lds_layout(std::max(h.sgs.total, h.sfs.total), h.cfg.rnn_dims, h.cfg.fc_dims).total *
           sizeof(float);
}

void pack_split_slabs(const wrnn_ctx &h, std::vector<float> &gs, std::vector<float> &fs) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, A = h.cfg.aux_dims, NC = h.cfg.n_classes;
    constexpr int U = kSplitUnits, NF = kSplitFcRows;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    const float *IW = W("I.weight");
    const int nin = 1 + h.cfg.feat_dims + A;
    const SplitGruSlab &sg = h.sgs;
    const SplitFcSlab &sf = h.sfs;
    gs.assign((size_t)h.sGg * sg.total, 0.0f);
    fs.assign((size_t)h.sGf * sf.total, 0.0f);
    std::vector<float> q1a(3 * R);
    for (int r = 0; r < 3 * R; ++r) q1a[r] = xcol_dot(W("rnn1.weight_ih_l0") + (size_t)r * R, IW, nin, R);
    for (int w = 0; w < h.sGg; ++w) {
        float *out = gs.data() + (size_t)w * sg.total;
        std::memcpy(out + sg.b3, W("fc3.bias"), (size_t)NC * 4);
        std::memcpy(out + sg.q1a, q1a.data(), (size_t)3 * R * 4);
        for (int u = 0; u < U; ++u) {
            const int j = w * U + u;
            out[sg.wi0 + u] = IW[(size_t)j * nin];
            for (int q = 0; q < 3; ++q) {
                const int src = q * R + j, dst = u * 3 + q;
                const float *ih2 = W("rnn2.weight_ih_l0") + (size_t)src * (R + A);
                std::memcpy(out + sg.wih2 + (size_t)dst * R, ih2, R * 4);
                std::memcpy(out + sg.whh1 + (size_t)dst * R, W("rnn1.weight_hh_l0") + (size_t)src * R, R * 4);
                std::memcpy(out + sg.whh2 + (size_t)dst * R, W("rnn2.weight_hh_l0") + (size_t)src * R, R * 4);
                out[sg.q2 + dst] = xcol_dot(ih2, IW, nin, R);
                out[sg.bih1 + dst] = W("rnn1.bias_ih_l0")[src];
                out[sg.bhh1 + dst] = W("rnn1.bias_hh_l0")[src];
                out[sg.bih2 + dst] = W("rnn2.bias_ih_l0")[src];
                out[sg.bhh2 + dst] = W("rnn2.bias_hh_l0")[src];
            }
        }
    }
    for (int w = 0; w < h.sGf; ++w) {
        float *out = fs.data() + (size_t)w * sf.total;
        for (int e = 0; e < NF; ++e) {
            const int r = w * NF + e;
            for (int j = 0; j < NC; ++j) out[sf.w3p + e * kSplitLogitLine + j] = W("fc3.weight")[(size_t)j * F + r];
            std::memcpy(out + sf.w1 + (size_t)e * R, W("fc1.weight") + (size_t)r * (R + A), R * 4);
            std::memcpy(out + sf.w2 + (size_t)e * F, W("fc2.weight") + (size_t)r * (F + A), F * 4);
        }
    }
}

// Terms-GEMM weights [(Gg + Gf)·kSplitTerms][KX] against X = [cI | a2 a3 a4 | 1 0 0 0]
// (fatchord_split.h, SplitTerm)
void pack_split_terms_weights(const wrnn_ctx &h, std::vector<float> &Wt) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, A = h.cfg.aux_dims, KX = h.KX;
    constexpr int U = kSplitUnits, NF = kSplitFcRows;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    Wt.assign((size_t)(h.sGg + h.sGf) * kSplitTerms * KX, 0.0f);
    for (int w = 0; w < h.sGg; ++w)
        for (int u = 0; u < U; ++u) {
            const int j = w * U + u;
            for (int q = 0; q < 3; ++q) {
                const int src = q * R + j;
                float *p1 = Wt.data() + ((size_t)w * kSplitTerms + ST_P1 + u * 3 + q) * KX;
                float *p2 = Wt.data() + ((size_t)w * kSplitTerms + ST_P2 + u * 3 + q) * KX;
                std::memcpy(p1, W("rnn1.weight_ih_l0") + (size_t)src * R, R * 4);
                const float *ih2 = W("rnn2.weight_ih_l0") + (size_t)src * (R + A);
                std::memcpy(p2, ih2, R * 4);
                std::memcpy(p2 + R, ih2 + R, A * 4);                            // a2
            }
            Wt[((size_t)w * kSplitTerms + ST_CI + u) * KX + j] = 1.0f;          // cI_j itself
        }
    for (int f = 0; f < h.sGf; ++f)
        for (int e = 0; e < NF; ++e) {
            const int r = f * NF + e;
            float *v1 = Wt.data() + ((size_t)(h.sGg + f) * kSplitTerms + ST_V1 + e) * KX;
            float *v2 = Wt.data() + ((size_t)(h.sGg + f) * kSplitTerms + ST_V2 + e) * KX;
            std::memcpy(v1 + R + A, W("fc1.weight") + (size_t)r * (R + A) + R, A * 4);   // a3
            v1[R + 3 * A] = W("fc1.bias")[r];
            std::memcpy(v2 + R + 2 * A, W("fc2.weight") + (size_t)r * (F + A) + F, A * 4);   // a4
            v2[R + 3 * A] = W("fc2.bias")[r];
        }
}

// ---- XCD-resident kernel (fatchord_xcd.h): workgroup c of an XCD owns units and fc rows
// 16c..16c+15; wave w of it units / fc rows 16c + 2w + {0, 1}
void make_xcd_slab(wrnn_ctx &h) {
    const int R = h.cfg.rnn_dims;
    int o = 0;
    auto take = [&](int n) { int at = o; o += round4(n); return at; };
    XcdSlab &x = h.xs;
    x.wih2 = take(kXWaves * 6 * R);
    x.w1 = take(kXWaves * 2 * R);
    x.w2 = take(kXWaves * 2 * R);
    x.whh2 = take(48 * R);
    x.whh1 = take(48 * R);
    x.w3 = take(kXWaves * 2 * 32);
    x.q1a = take(3 * R);
    x.cst = take(kXCst);
    x.total = o;
}

void pack_xcd_slab(const wrnn_ctx &h, std::vector<float> &slab) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, A = h.cfg.aux_dims, NC = h.cfg.n_classes;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    const float *IW = W("I.weight");
    const int nin = 1 + h.cfg.feat_dims + A;
    const XcdSlab &x = h.xs;
    slab.assign((size_t)kXcdWgs * x.total, 0.0f);
    std::vector<float> q1a(3 * R);
    for (int r = 0; r < 3 * R; ++r) q1a[r] = xcol_dot(W("rnn1.weight_ih_l0") + (size_t)r * R, IW, nin, R);
    for (int c = 0; c < kXcdWgs; ++c) {
        float *out = slab.data() + (size_t)c * x.total;
        std::memcpy(out + x.q1a, q1a.data(), (size_t)3 * R * 4);
        for (int w = 0; w < kXWaves; ++w)
            for (int i = 0; i < 2; ++i) {
                const int u = 2 * w + i, j = c * kXUnits + u;     // unit j, fc row j
                for (int q = 0; q < 3; ++q)
                    std::memcpy(out + x.wih2 + (size_t)(w * 6 + 2 * q + i) * R,
                                W("rnn2.weight_ih_l0") + (size_t)(q * R + j) * (R + A), R * 4);
                std::memcpy(out + x.w1 + (size_t)(w * 2 + i) * R, W("fc1.weight") + (size_t)j * (R + A), R * 4);
                std::memcpy(out + x.w2 + (size_t)(w * 2 + i) * R, W("fc2.weight") + (size_t)j * (F + A), F * 4);
                for (int k = 0; k < NC; ++k) out[x.w3 + (w * 2 + i) * 32 + k] = W("fc3.weight")[(size_t)k * F + j];
            }
        for (int u = 0; u < kXUnits; ++u) {
            const int j = c * kXUnits + u;
            out[x.cst + XC_WI0 + u] = IW[(size_t)j * nin];
            for (int q = 0; q < 3; ++q) {
                const int src = q * R + j, rr = u * 3 + q;
                std::memcpy(out + x.whh1 + (size_t)rr * R, W("rnn1.weight_hh_l0") + (size_t)src * R, R * 4);
                std::memcpy(out + x.whh2 + (size_t)rr * R, W("rnn2.weight_hh_l0") + (size_t)src * R, R * 4);
                out[x.cst + XC_Q2 + rr] = xcol_dot(W("rnn2.weight_ih_l0") + (size_t)src * (R + A), IW, nin, R);
                out[x.cst + XC_BIH1 + rr] = W("rnn1.bias_ih_l0")[src];
                out[x.cst + XC_BHH1 + rr] = W("rnn1.bias_hh_l0")[src];
                out[x.cst + XC_BIH2 + rr] = W("rnn2.bias_ih_l0")[src];
                out[x.cst + XC_BHH2 + rr] = W("rnn2.bias_hh_l0")[src];
            }
        }
        for (int k = 0; k < NC; ++k) out[x.cst + XC_B3 + k] = W("fc3.bias")[k];
    }
}

// The XCD kernels' terms-GEMM rows against X' = [mel | a1 | a2 | a3 | a4 | 1 0 0 0] (KXc = CD + 4):
// the I layer (fatchord_version.py:208, cI = W_I·[mel; a1] + b_I; the x column is folded
// separately, q1a / q2) is composed into the W_ih1 / W_ih2 rows in fp64 here, so the GEMM runs on
// the 208-wide conditioning record instead of a 900-wide cI (4.7x less work at rnn 896).
void fold_ci_row(const wrnn_ctx &h, const float *w, float *dst) {
    const int R = h.cfg.rnn_dims, M = h.cfg.feat_dims, A = h.cfg.aux_dims, nin = 1 + M + A;
    const float *IW = h.w.at("I.weight").data(), *Ib = h.w.at("I.bias").data();
    std::vector<double> acc(M + A + 1, 0.0);
    for (int k = 0; k < R; ++k) {
        const double wk = w[k];
        if (wk == 0.0) continue;
        const float *iw = IW + (size_t)k * nin + 1;
        for (int m = 0; m < M + A; ++m) acc[m] += wk * iw[m];
        acc[M + A] += wk * Ib[k];
    }
    for (int m = 0; m < M + A; ++m) dst[m] += (float)acc[m];
    dst[h.CD] += (float)acc[M + A];
}

// slot rows of one unit j (gates q = 0..2: p1q[q], p2q[q]; its cI: ci) and of one fc row r
// (v1, v2) for the composed input X'
void pack_xcd_unit_terms(const wrnn_ctx &h, int j, float *const p1q[3], float *const p2q[3], float *ci) {
    const int R = h.cfg.rnn_dims, M = h.cfg.feat_dims, A = h.cfg.aux_dims, nin = 1 + M + A;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    for (int q = 0; q < 3; ++q) {
        const int src = q * R + j;
        fold_ci_row(h, W("rnn1.weight_ih_l0") + (size_t)src * R, p1q[q]);
        const float *ih2 = W("rnn2.weight_ih_l0") + (size_t)src * (R + A);
        fold_ci_row(h, ih2, p2q[q]);
        for (int a = 0; a < A; ++a) p2q[q][M + A + a] += ih2[R + a];                      // a2
    }
    const float *iw = W("I.weight") + (size_t)j * nin + 1;
    for (int m = 0; m < M + A; ++m) ci[m] = iw[m];                                         // cI_j
    ci[h.CD] = W("I.bias")[j];
}
void pack_xcd_fc_terms(const wrnn_ctx &h, int r, float *v1, float *v2) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, M = h.cfg.feat_dims, A = h.cfg.aux_dims;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    for (int a = 0; a < A; ++a) {
        v1[M + 2 * A + a] = W("fc1.weight")[(size_t)r * (R + A) + R + a];                 // a3
        v2[M + 3 * A + a] = W("fc2.weight")[(size_t)r * (F + A) + F + a];                 // a4
    }
    v1[h.CD] = W("fc1.bias")[r];
    v2[h.CD] = W("fc2.bias")[r];
}

// Terms-GEMM weights [kXcdWgs·kXTerms][KXc] (XTerm slots) against X'
void pack_xcd_terms_weights(const wrnn_ctx &h, std::vector<float> &Wt) {
    const int KX = h.KXc;
    Wt.assign((size_t)kXcdWgs * kXTerms * KX, 0.0f);
    for (int c = 0; c < kXcdWgs; ++c) {
        auto row = [&](int slot) { return Wt.data() + ((size_t)c * kXTerms + slot) * KX; };
        for (int u = 0; u < kXUnits; ++u) {
            float *const p1q[3] = {row(XT_P1 + u * 3), row(XT_P1 + u * 3 + 1), row(XT_P1 + u * 3 + 2)};
            float *const p2q[3] = {row(XT_P2 + u * 3), row(XT_P2 + u * 3 + 1), row(XT_P2 + u * 3 + 2)};
            pack_xcd_unit_terms(h, c * kXUnits + u, p1q, p2q, row(XT_CI + u));
            pack_xcd_fc_terms(h, c * kXUnits + u, row(XT_V1 + u), row(XT_V2 + u));
        }
    }
}

// Many-row kernel: its compact terms record (kMRing slots per workgroup, MT_ order) segmented by
// GEMM group (fatchord_xcdm.h, mterm_off) with the columns in the split input order X'' = [mel |
// a1 | 1 | a2 | a3 | a4 | 1 | 0 0] (pack_cond_input_kernel, split = M + A): P1 and cI depend on
// mel‖a1 and their bias only, P2 also on a2, V1 / V2 on a3 / a4 and their biases — generate_xcdm
// runs one GEMM per group over just those columns (xcdm_terms_gemms).
void pack_xcdm_terms_weights(const wrnn_ctx &h, std::vector<float> &Wm) {
    std::vector<float> Wt;
    pack_xcd_terms_weights(h, Wt);
    const int KX = h.KXc, CD = h.CD, split = h.cfg.feat_dims + h.cfg.aux_dims;
    Wm.assign((size_t)kXcdWgs * kMRing * KX, 0.0f);
    for (int c = 0; c < kXcdWgs; ++c)
        for (int s = 0; s < kMRing; ++s) {
            const float *src = Wt.data() + ((size_t)c * kXTerms + mterm_xt(s)) * KX;
            float *dst = Wm.data() + (size_t)mterm_off(c, s) * KX;
            for (int j = 0; j < CD; ++j) dst[j < split ? j : j + 1] = src[j];
            dst[s >= MT_V1 ? CD + 1 : split] = src[CD];          // the bias → its group's ones column
        }
}

// (record rows, first input column, depth) of each group: [P1 | cI] on mel‖a1‖1, P2 on
// mel‖a1‖1‖a2, [V1 | V2] on a3‖a4‖1 — depths rounded up to a multiple of 4 over zero weights
struct XcdmGemm {
    int row0, rows, col0, k;
};
void xcdm_terms_gemms(const wrnn_ctx &h, XcdmGemm (&g)[3]) {
    const int M = h.cfg.feat_dims, A = h.cfg.aux_dims, split = M + A;
    auto up4 = [](int n) { return (n + 3) / 4 * 4; };
    const int v0 = (split + 1 + A) / 4 * 4;                     // first column of a3, rounded down
    g[0] = {kMG0, kMG1 - kMG0, 0, std::min(up4(split + 1), h.KXc)};
    g[1] = {kMG1, kMG2 - kMG1, 0, std::min(up4(split + 1 + A), h.KXc)};
    g[2] = {kMG2, kMGEnd - kMG2, v0, std::min(up4(h.CD + 2 - v0), h.KXc - v0)};
}

// ---- XCD-resident block-sparse kernel (fatchord_xcds.h): workgroup c of an XCD owns units
// 28c..28c+27 (block-rows ub = 0..6 of each gate) and fc rows 16c..16c+15
void make_xcds_slab(wrnn_ctx &h) {
    int o = 0;
    auto take = [&](int n) { int at = o; o += round4(n); return at; };
    XcdsSlab &x = h.xss;
    x.wih2b = take(kSBR * kSNB * 16);
    x.whh1b = take(kSBR * kSNB * 16);
    x.whh2b = take(kSBR * kSNB * 16);
    x.wih2c = take(kSBR * kSNB);
    x.whh1c = take(kSBR * kSNB);
    x.whh2c = take(kSBR * kSNB);
    x.w1 = take(kXFcRows * kSR);
    x.w2 = take(kXFcRows * 512);
    x.w3 = take(kXFcRows * 32);
    x.q1a = take(3 * kSR);
    x.cst = take(kSCst);
    x.total = o;
}

// nonzero 4x4 blocks of the gate block-row (q, 4-unit group u4) of a loop matrix
std::vector<int> xcds_blocks(const LoopMat &m, int q, int u4) {
    std::vector<int> cols;
    for (int cb = 0; cb < kSR; cb += 4)
        if (block_nonzero(m.w, m.ld, q * kSR + 4 * u4, cb)) cols.push_back(cb / 4);
    return cols;
}

// largest nonzero-block count over every gate block-row of W_ih2[:, :R], W_hh1, W_hh2
int xcds_nbmax(const wrnn_ctx &h) {
    LoopMat m[3];
    loop_mats(h, m);
    int mx = 0;
    for (int k = 0; k < 3; ++k)
        for (int q = 0; q < 3; ++q)
            for (int u4 = 0; u4 < kSR / 4; ++u4) mx = std::max(mx, (int)xcds_blocks(m[k], q, u4).size());
    return mx;
}

void pack_xcds_slab(const wrnn_ctx &h, std::vector<float> &slab) {
    const int R = kSR, F = h.cfg.fc_dims, A = h.cfg.aux_dims, NC = h.cfg.n_classes;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    const float *IW = W("I.weight");
    const int nin = 1 + h.cfg.feat_dims + A;
    const XcdsSlab &x = h.xss;
    slab.assign((size_t)kXcdWgs * x.total, 0.0f);
    std::vector<float> q1a(3 * R);
    for (int r = 0; r < 3 * R; ++r) q1a[r] = xcol_dot(W("rnn1.weight_ih_l0") + (size_t)r * R, IW, nin, R);
    LoopMat m[3];
    loop_mats(h, m);
    const int boff[3] = {x.wih2b, x.whh1b, x.whh2b}, coff[3] = {x.wih2c, x.whh1c, x.whh2c};
    for (int c = 0; c < kXcdWgs; ++c) {
        float *out = slab.data() + (size_t)c * x.total;
        std::memcpy(out + x.q1a, q1a.data(), (size_t)3 * R * 4);
        for (int k = 0; k < 3; ++k)
            for (int q = 0; q < 3; ++q)
                for (int ub = 0; ub < kSUB; ++ub) {
                    const int br = q * kSUB + ub, u4 = c * kSUB + ub, r0 = q * R + 4 * u4;
                    const std::vector<int> cols = xcds_blocks(m[k], q, u4);
                    int *cc = reinterpret_cast<int *>(out + coff[k]) + br * kSNB;
                    for (size_t n = 0; n < cols.size() && n < (size_t)kSNB; ++n) {
                        float *blk = out + boff[k] + ((size_t)br * kSNB + n) * 16;
                        for (int r = 0; r < 4; ++r)
                            for (int cc4 = 0; cc4 < 4; ++cc4)
                                blk[r * 4 + cc4] = m[k].w[(size_t)(r0 + r) * m[k].ld + 4 * cols[n] + cc4];
                        cc[n] = cols[n];
                    }
                }
        for (int r = 0; r < kXFcRows; ++r) {
            const int j = c * kXFcRows + r;
            std::memcpy(out + x.w1 + (size_t)r * R, W("fc1.weight") + (size_t)j * (R + A), R * 4);
            std::memcpy(out + x.w2 + (size_t)r * F, W("fc2.weight") + (size_t)j * (F + A), F * 4);
            for (int kk = 0; kk < NC; ++kk) out[x.w3 + r * 32 + kk] = W("fc3.weight")[(size_t)kk * F + j];
        }
        for (int u = 0; u < kSU; ++u) {
            const int j = c * kSU + u;
            out[x.cst + SC_WI0 + u] = IW[(size_t)j * nin];
            for (int q = 0; q < 3; ++q) {
                const int src = q * R + j, rr = u * 3 + q;
                out[x.cst + SC_Q2 + rr] = xcol_dot(W("rnn2.weight_ih_l0") + (size_t)src * (R + A), IW, nin, R);
                out[x.cst + SC_BIH1 + rr] = W("rnn1.bias_ih_l0")[src];
                out[x.cst + SC_BHH1 + rr] = W("rnn1.bias_hh_l0")[src];
                out[x.cst + SC_BIH2 + rr] = W("rnn2.bias_ih_l0")[src];
                out[x.cst + SC_BHH2 + rr] = W("rnn2.bias_hh_l0")[src];
            }
        }
        for (int kk = 0; kk < NC; ++kk) out[x.cst + SC_B3 + kk] = W("fc3.bias")[kk];
    }
}

// Terms-GEMM weights [kXcdWgs·kSTerms][KXc] (SXTerm slots) against X' (pack_xcd_terms_weights)
void pack_xcds_terms_weights(const wrnn_ctx &h, std::vector<float> &Wt) {
    const int KX = h.KXc;
    Wt.assign((size_t)kXcdWgs * kSTerms * KX, 0.0f);
    for (int c = 0; c < kXcdWgs; ++c) {
        auto row = [&](int slot) { return Wt.data() + ((size_t)c * kSTerms + slot) * KX; };
        for (int u = 0; u < kSU; ++u) {
            float *const p1q[3] = {row(SX_P1 + u * 3), row(SX_P1 + u * 3 + 1), row(SX_P1 + u * 3 + 2)};
            float *const p2q[3] = {row(SX_P2 + u * 3), row(SX_P2 + u * 3 + 1), row(SX_P2 + u * 3 + 2)};
            pack_xcd_unit_terms(h, c * kSU + u, p1q, p2q, row(SX_CI + u));
        }
        for (int r = 0; r < kXFcRows; ++r) pack_xcd_fc_terms(h, c * kXFcRows + r, row(SX_V1 + r), row(SX_V2 + r));
    }
}

// ---- XCD-resident many-row kernel (fatchord_xcdm.h): per workgroup c the MFMA A operands of the
// eleven 16-row sets (wave w: K window [kMK·w, kMK·(w + 1))), the fc3 columns of its f2 rows and
// the small vectors
void make_xcdm_slab(wrnn_ctx &h) {
    int o = 0;
    auto take = [&](int n) { int at = o; o += round4(n); return at; };
    XcdmSlab &x = h.xms;
    const bool raw = h.cfg.mode == WRNN_MODE_RAW;
    x.a = take(kMWaves * kMSets * kMJ * 64);
    x.a3 = take(raw ? kMWaves * kMJ * 64 : 0);
    x.w3 = take(raw ? 0 : 32 * kMW3Stride);
    x.cst = take(kMCst);
    x.total = o;
}

void pack_xcdm_slab(const wrnn_ctx &h, std::vector<float> &slab) {
    const int R = h.cfg.rnn_dims, F = h.cfg.fc_dims, A = h.cfg.aux_dims, NC = h.cfg.n_classes;
    auto W = [&](const char *n) { return h.w.at(n).data(); };
    const float *IW = W("I.weight");
    const int nin = 1 + h.cfg.feat_dims + A;
    const XcdmSlab &x = h.xms;
    slab.assign((size_t)kXcdWgs * x.total, 0.0f);
    // row r (0..15) of set s of workgroup c: (matrix, row index, row stride)
    auto set_row = [&](int s, int c, int r) -> const float * {
        if (s < MS_FC1) return W("rnn2.weight_ih_l0") + (size_t)(s * R + 16 * c + r) * (R + A);
        if (s == MS_FC1) return W("fc1.weight") + (size_t)(16 * c + r) * (R + A);
        if (s == MS_FC2) return W("fc2.weight") + (size_t)(16 * c + r) * (F + A);
        if (s < MS_HH1) return W("rnn2.weight_hh_l0") + (size_t)((s - MS_HH2) * R + 16 * c + r) * R;
        return W("rnn1.weight_hh_l0") + (size_t)((s - MS_HH1) * R + 16 * c + r) * R;
    };
    for (int c = 0; c < kXcdWgs; ++c) {
        float *out = slab.data() + (size_t)c * x.total;
        for (int w = 0; w < kMWaves; ++w)
            for (int s = 0; s < kMSets; ++s)
                for (int j = 0; j < kMJ; ++j)
                    for (int l = 0; l < 64; ++l) {
                        const int g = (l >> 2) & 3, sp = l >> 4, j4 = l & 3;
                        out[x.a + (((size_t)w * kMSets + s) * kMJ + j) * 64 + l] =
                            set_row(s, c, 4 * g + j4)[kMK * w + kMJ * sp + j];
                    }
        if (h.cfg.mode == WRNN_MODE_RAW) {   // fc3 rows of the own classes 16c + r, [wave][k-chunk][lane][4]
            for (int w = 0; w < kMWaves; ++w)
                for (int j = 0; j < kMJ; ++j)
                    for (int l = 0; l < 64; ++l)
                        out[x.a3 + ((size_t)(w * (kMJ / 4) + j / 4) * 64 + l) * 4 + (j & 3)] =
                            W("fc3.weight")[(size_t)(16 * c + (l & 15)) * F + kMK * w + kMJ * (l >> 4) + j];
        } else {
            for (int jj = 0; jj < NC; ++jj)
                for (int r = 0; r < 16; ++r) out[x.w3 + jj * kMW3Stride + r] = W("fc3.weight")[(size_t)jj * F + 16 * c + r];
        }
        for (int u = 0; u < 16; ++u) {
            const int j = 16 * c + u;
            out[x.cst + MC_WI0 + u] = IW[(size_t)j * nin];
            for (int q = 0; q < 3; ++q) {
                const int src = q * R + j, i = q * 16 + u;
                out[x.cst + MC_Q1 + i] = xcol_dot(W("rnn1.weight_ih_l0") + (size_t)src * R, IW, nin, R);
                out[x.cst + MC_Q2 + i] = xcol_dot(W("rnn2.weight_ih_l0") + (size_t)src * (R + A), IW, nin, R);
                out[x.cst + MC_BIH1 + i] = W("rnn1.bias_ih_l0")[src];
                out[x.cst + MC_BHH1 + i] = W("rnn1.bias_hh_l0")[src];
                out[x.cst + MC_BIH2 + i] = W("rnn2.bias_ih_l0")[src];
                out[x.cst + MC_BHH2 + i] = W("rnn2.bias_hh_l0")[src];
            }
        }
        if (h.cfg.mode == WRNN_MODE_RAW)
            for (int r = 0; r < 16; ++r) out[x.cst + MC_B3 + r] = W("fc3.bias")[16 * c + r];
        else
            for (int jj = 0; jj < NC; ++jj) out[x.cst + MC_B3 + jj] = W("fc3.bias")[jj];
    }
}

}  // namespace

namespace {

// grow-only device buffer
template <typename T>
hipError_t ensure(T *&p, size_t &cap, size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) {
        hipError_t e = hipFree(p);
        if (e != hipSuccess) return e;
    }
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
}

// WRNN_DEBUG_STAMPS buffer: freed on every exit path (an early HIP_TRY / fail() return included);
// the dump helpers take ownership by resetting p first
struct DbgBuf {
    unsigned *p = nullptr;
    DbgBuf() = default;
    DbgBuf(const DbgBuf &) = delete;
    DbgBuf &operator=(const DbgBuf &) = delete;
    ~DbgBuf() {
        if (p) (void)hipFree(p);
    }
    unsigned *release() {
        unsigned *q = p;
        p = nullptr;
        return q;
    }
};

// per-wave stamps of the many-row / deepmind kernels: int32 header {waves, steps, stamps}
int dump_wave_stamps(wrnn_t *h, DbgBuf &dbg, size_t n, int waves, int steps, int stamps, hipStream_t st) {
    std::vector<unsigned> host(n);
    HIP_TRY(h, hipStreamSynchronize(st));
    HIP_TRY(h, hipMemcpy(host.data(), dbg.p, n * 4, hipMemcpyDeviceToHost));
    HIP_TRY(h, hipFree(dbg.release()));
    const char *path = std::getenv("WRNN_DEBUG_FILE");
    if (FILE *f = std::fopen(path ? path : "wrnn_stamps.bin", "wb")) {
        int hdr[3] = {waves, steps, stamps};
        std::fwrite(hdr, sizeof(hdr), 1, f);
        std::fwrite(host.data(), 4, host.size(), f);
        std::fclose(f);
    }
    return WRNN_OK;
}

// WRNN_DEBUG_FILE (default wrnn_stamps.bin): int32 header {G, steps, kStamps}, then the stamps
int dump_stamps(wrnn_t *h, unsigned *d_dbg, int dbg_steps, hipStream_t st, int G) {
    std::vector<unsigned> host((size_t)G * dbg_steps * kStamps);
    HIP_TRY(h, hipStreamSynchronize(st));
    HIP_TRY(h, hipMemcpy(host.data(), d_dbg, host.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(h, hipFree(d_dbg));
    const char *path = std::getenv("WRNN_DEBUG_FILE");
    if (FILE *f = std::fopen(path ? path : "wrnn_stamps.bin", "wb")) {
        int hdr[3] = {G, dbg_steps, kStamps};
        std::fwrite(hdr, sizeof(hdr), 1, f);
        std::fwrite(host.data(), 4, host.size(), f);
        std::fclose(f);
    }
    return WRNN_OK;
}

int grow(wrnn_t *h, float *&p, size_t &cap, size_t n) {
    HIP_TRY(h, ensure(p, cap, n));
    return WRNN_OK;
}

// B rows through the multi-row kernel: row blocks of <= kRowsMax rows per launch, time chunks
// sized so the precomputed terms stay within WRNN_TERMS_MB (default 8192 MiB).  Blocks of
// >= kGroupRows rows run as two row groups of half the rows on G/2 workgroups each (the grouped
// partition, dense weights only; WRNN_ROW_GROUPS=1|2 forces one or the other).  Measured on
// MI355X (MoL 512, us/step, one group → two): B=2 17.2 → 15.7, B=10 18.3 → 16.9, B=32 26.6 →
// 19.5, B=115 51.2 → 40.2: half the rows streamed per stage and half the flags per hop.
constexpr int kGroupRows = 2;
constexpr size_t kRowsGranMax = 4096;   // values per row group and hop up to which hops use granules
constexpr size_t kDmGranMax = 8192;     // the same for the deepmind kernel (one poll round of all waves)

int generate_rows(wrnn_t *h, const float *cond, int B, int L, const float *noise, uint64_t seed, int64_t row_offset,
                  float *out, int32_t *labels, hipStream_t st) {
    const wrnn_config &c = h->cfg;
    const char *gran_env = std::getenv("WRNN_ROWS_GRANULES");
    const int gran_force = gran_env ? std::atoi(gran_env) : -1;
    const char *grp_env = std::getenv("WRNN_ROW_GROUPS");
    const int grp_force = grp_env ? std::atoi(grp_env) : 0;
    const bool can_group = h->g2.ok && !h->sparse && grp_force != 1;
    const bool grouped = can_group && B >= 2 && (grp_force == 2 || std::min(B, kRowsMax) >= kGroupRows);
    PartScope ps(*h, h->g2, grouped);          // h->r*, rs, NT, d_rslab, d_Wt = the grouped partition
    const int ng = grouped ? 2 : 1;
    const int R = c.rnn_dims, A = c.aux_dims, N = h->rG * h->NT;
    const size_t flag_words = (size_t)kRowsHops * kFlagSlots * kFlagStride, xr_words = (size_t)kXReps * kXRepStride;
    if (!h->d_flags) {
        HIP_TRY(h, hipMalloc(&h->d_flags, 2 * flag_words * 4));
        HIP_TRY(h, hipMalloc(&h->d_xr, 2 * xr_words * 8));
    }
    if (!h->blas && rocblas_create_handle(&h->blas) != rocblas_status_success)
        return fail(h, WRNN_EHIP, "rocblas_create_handle failed");
    if (rocblas_set_stream(h->blas, st) != rocblas_status_success) return fail(h, WRNN_EHIP, "rocblas_set_stream failed");
    const char *mb_env = std::getenv("WRNN_TERMS_MB");
    const double budget = (mb_env ? std::atof(mb_env) : 8192.0) * (1 << 20) / 4.0;   // floats
    const float one = 1.0f, zero = 0.0f;
    const char *dbg_env = std::getenv("WRNN_DEBUG_STAMPS");
    const int dbg_steps = dbg_env ? std::min(L, std::atoi(dbg_env)) : 0;
    DbgBuf dbg;
    if (dbg_steps > 0) {
        HIP_TRY(h, hipMalloc(&dbg.p, (size_t)h->rG * dbg_steps * kStamps * 4));
        HIP_TRY(h, hipMemsetAsync(dbg.p, 0, (size_t)h->rG * dbg_steps * kStamps * 4, st));
    }
    for (int b0 = 0; b0 < B;) {
        int Bl = std::min(B - b0, kRowsMax);
        auto group_rows = [&](int bl, int g) { const int b_0 = (bl + ng - 1) / ng; return g == 0 ? b_0 : bl - b_0; };
        while (Bl > 1 && rows_tile_for(*h, group_rows(Bl, 0)) == 0 && rows_tile_for(*h, group_rows(Bl, 0), false) == 0) --Bl;
        const int Bg = group_rows(Bl, 0);          // rows of group 0 (>= those of group 1)
        // the MoL head stays in LDS while all rows fit one tile next to it; beyond that, larger
        // tiles are worth more than an LDS-resident head (the samplers then read it from L2)
        const bool mol = c.mode == WRNN_MODE_MOL;
        const int tb_in = rows_tile_for(*h, Bg);
        const bool head_lds = !mol || tb_in >= std::min(Bg, 16) || rows_tile_for(*h, Bg, false) == 0;
        const int TB = head_lds ? tb_in : rows_tile_for(*h, Bg, false);
        if (TB == 0) return fail(h, WRNN_EUNSUPPORTED, "rows kernel: one row of state does not fit LDS");
        const int SW = rows_state_width(h->rU, h->rUF);
        // GEMM input width: the composed MoL record (KXc = CD + 4) or [cI | a2 a3 a4 | 1 0 0 0]
        // (KX); either may be the larger one (tiny dims: KXc 100 > KX 80)
        const int KXg = rows_terms_kx(*h);
        const int Lc_max = (int)std::max(1.0, std::min((double)L, budget / ((double)Bl * (N + KXg))));
        const size_t T_grp = (size_t)Lc_max * Bg * N, act_grp = (size_t)kRowsHops * 2 * Bg * h->KA;
        const size_t state_grp = (size_t)h->rG * Bg * SW + Bg;
        if (grow(h, h->d_X, h->X_cap, (size_t)Lc_max * Bg * KXg) || grow(h, h->d_T, h->T_cap, ng * T_grp) ||
            grow(h, h->d_act, h->act_cap, ng * act_grp) || grow(h, h->d_state, h->state_cap, ng * state_grp))
            return WRNN_EHIP;
        HIP_TRY(h, hipMemsetAsync(h->d_flags, 0, ng * flag_words * 4, st));
        HIP_TRY(h, hipMemsetAsync(h->d_xr, 0, ng * xr_words * 8, st));
        // granule hand-offs while a group's hop vector is small (kRowsGranMax values; measured
        // crossover); WRNN_ROWS_GRANULES=0|1 forces bulk / granules.  The granules
        // are zeroed per row block: tags restart at 1 with every generate()
        const bool gran = gran_force == 1 || (gran_force != 0 && (size_t)Bg * h->KA <= kRowsGranMax);
        const long long gstride = (((long long)Bg * h->KA + kRowsGranPad + 15) / 16) * 16;
        // bulk mode, MoL: the f2 hop alone as granules (one hop region per group)
        const bool f2g = !gran && mol;
        if (gran || f2g) {
            const size_t n = (size_t)ng * (gran ? kRowsHops : 1) * gstride;
            HIP_TRY(h, ensure(h->d_gact, h->gact_cap, n));
            HIP_TRY(h, hipMemsetAsync(h->d_gact, 0, n * 8, st));
        }
        for (int t0 = 0; t0 < L; t0 += Lc_max) {
            const int Lc = std::min(Lc_max, L - t0);
            // conditioning terms of steps [t0, t0 + Lc), per group: cI, then one fp32 GEMM for
            // every workgroup's terms
            for (int g = 0; g < ng; ++g) {
                const int bg0 = b0 + (g ? Bg : 0), nb = group_rows(Bl, g);
                if ((size_t)Lc * nb * KXg > h->X_cap) return fail(h, WRNN_EINVAL, "terms-GEMM input exceeds its workspace");
                if (rows_terms_composed(*h)) {
                    HIP_TRY(h, launch_pack_cond_input(cond, h->CD, B, bg0, nb, t0, Lc, KXg, h->d_X, st));
                } else {
                    HIP_TRY(h, launch_ci_gemm(cond, h->CD, B, bg0, nb, t0, Lc, h->d_IW, 1 + c.feat_dims + A, h->d_Ib, R,
                                              c.feat_dims + A, h->d_X, h->KX, st));
                    HIP_TRY(h, launch_pack_terms_input(cond, h->CD, B, bg0, nb, t0, Lc, c.feat_dims, A, R, h->KX, h->d_X, st));
                }
                if (rocblas_sgemm(h->blas, rocblas_operation_transpose, rocblas_operation_none, N, Lc * nb, KXg, &one,
                                  h->d_Wt, KXg, h->d_X, KXg, &zero, h->d_T + g * T_grp, N) != rocblas_status_success)
                    return fail(h, WRNN_EHIP, "rocblas_sgemm (conditioning terms) failed");
            }
            RowsArgs a{};
            a.slab = h->d_rslab;
            a.terms = h->d_T;
            a.noise = noise;
            a.out = out;
            a.labels = labels;
            a.act = h->d_act;
            a.flags = h->d_flags;
            a.xg = h->d_xr;
            a.gact = gran ? h->d_gact : nullptr;
            a.gstride = gstride;
            a.gf2 = f2g ? h->d_gact : nullptr;
            a.state = h->d_state;
            a.ctl = h->d_ctl;
            a.seed = seed;
            a.row0 = row_offset + b0;
            a.timeout_ticks = h->timeout_ticks;
            a.L = L;
            a.t0 = t0;
            a.Lc = Lc;
            a.B = Bg;
            a.Bt = B;
            a.b0 = b0;
            a.R = R;
            a.F = c.fc_dims;
            a.A = A;
            a.NC = c.n_classes;
            a.NK = h->NK;
            a.mol = c.mode == WRNN_MODE_MOL;
            a.U = h->rU;
            a.UF = h->rUF;
            a.UC = h->rUC;
            a.G = h->rG;
            a.NT = h->NT;
            a.TB = TB;
            a.KA = h->KA;
            a.s = h->rs;
            a.dbg = (b0 == 0 && t0 == 0) ? dbg.p : nullptr;
            a.dbg_steps = std::min(dbg_steps, Lc);
            a.head_lds = head_lds ? 1 : 0;
            a.gw = h->rows_gw ? 1 : 0;
            RowsGroup g1{};
            if (grouped) {
                g1.terms = h->d_T + T_grp;
                g1.act = h->d_act + act_grp;
                g1.flags = h->d_flags + flag_words;
                g1.xg = h->d_xr + xr_words;
                g1.gact = gran ? h->d_gact + (size_t)kRowsHops * gstride : nullptr;
                g1.gf2 = f2g ? h->d_gact + gstride : nullptr;
                g1.state = h->d_state + state_grp;
                g1.row0 = row_offset + b0 + Bg;
                g1.B = group_rows(Bl, 1);
                g1.b0 = b0 + Bg;
                g1.dbg = nullptr;
            }
            HIP_TRY(h, launch_rows(a, grouped ? &g1 : nullptr, rows_lds_bytes(*h, Bg, TB, head_lds), st));
        }
        b0 += Bl;
    }
    if (dbg.p) return dump_stamps(h, dbg.release(), dbg_steps, st, h->rG);
    return WRNN_OK;
}

// deepmind_version: B rows (utterances) in row groups of <= kRowsMax, one launch each
// deepmind rows through the XCD-resident kernel: up to kDxRowsMax rows per launch (launch row r
// on XCD r % 8); Philox draws precomputed per time chunk (≤ WRNN_DM_NOISE_MB, default 2 GiB: config
// 5's 32 rows × 16 000 steps are 1 GiB of draws, one fill and ONE persistent launch — with 64 MiB
// chunks the call was 16 launches, ≈ 0.24 µs per step of relaunch, prologue and fill; the draws of
// a step are read once per XCD, ≈ 10 GB/s from HBM, so they need not stay in the Infinity Cache);
// the recurrent state carried per workgroup in d_dxstate.
int generate_dx(wrnn_t *h, int B, int L, const float *noise, uint64_t seed, int64_t row_offset, float *out,
                int32_t *labels, hipStream_t st) {
    const size_t xg_words = (size_t)kXcds * kDxXcdStride;
    if (!h->d_members) HIP_TRY(h, hipMalloc(&h->d_members, kXcds * sizeof(int)));
    if (!h->d_dxxg) HIP_TRY(h, hipMalloc(&h->d_dxxg, xg_words * 8));
    if (!h->d_dxstate) HIP_TRY(h, hipMalloc(&h->d_dxstate, (size_t)kXcds * kXcdWgs * kDxStateW * sizeof(float)));
    const char *mb_env = std::getenv("WRNN_DM_NOISE_MB");
    const double budget = (mb_env ? std::atof(mb_env) : 2048.0) * (1 << 20) / 4.0;   // floats
    const char *dbg_env = std::getenv("WRNN_DEBUG_STAMPS");
    const int dbg_steps = (dbg_env && std::atoi(dbg_env) > 0 && L >= kDxDbgSkip + kDxDbgSteps) ? kDxDbgSteps : 0;
    const size_t dbg_n = (size_t)kXcds * kXcdWgs * kDxWaves * dbg_steps * kDxStamps;
    DbgBuf dbg;
    if (dbg_steps > 0) {
        HIP_TRY(h, hipMalloc(&dbg.p, dbg_n * 4));
        HIP_TRY(h, hipMemsetAsync(dbg.p, 0, dbg_n * 4, st));
    }
    for (int b0 = 0; b0 < B; b0 += kDxRowsMax) {
        const int nb = std::min(kDxRowsMax, B - b0);
        const int Lc_max = noise ? L : (int)std::max(1.0, std::min((double)L, budget / ((double)nb * 2 * kDxQ)));
        if (!noise && grow(h, h->d_dxnoise, h->dxnoise_cap, (size_t)Lc_max * nb * 2 * kDxQ)) return WRNN_EHIP;
        HIP_TRY(h, hipMemsetAsync(h->d_dxxg, 0, xg_words * 8, st));   // tags restart at 1
        for (int t0 = 0; t0 < L; t0 += Lc_max) {
            const int Lc = std::min(Lc_max, L - t0);
            HIP_TRY(h, hipMemsetAsync(h->d_members, 0, kXcds * sizeof(int), st));
            DxArgs a{};
            a.slab = h->d_dxslab;
            if (noise) {   // injected [L][B][2Q]
                a.noise = noise;
                a.nz_t0 = 0;
                a.nz_ts = B;
                a.nz_b0 = b0;
            } else {       // Philox Exp(1) draws of this chunk ([Lc][nb][2Q]), keyed as every kernel keys them
                HIP_TRY(h, launch_philox_fill(h->d_dxnoise, seed, row_offset + b0, nb, t0, Lc, 2 * kDxQ, 0, st));
                a.noise = h->d_dxnoise;
                a.nz_t0 = t0;
                a.nz_ts = nb;
                a.nz_b0 = 0;
            }
            a.out = out;
            a.labels = labels;
            a.state = h->d_dxstate;
            a.xg = h->d_dxxg;
            a.members = h->d_members;
            a.ctl = h->d_ctl;
            a.timeout_ticks = h->timeout_ticks;
            a.L = L;
            a.t0 = t0;
            a.Lc = Lc;
            a.Bt = B;
            a.b0 = b0;
            a.nb = nb;
            a.s = dx_slab_layout();
            a.dbg = (b0 == 0 && t0 == 0 && Lc >= kDxDbgSkip + kDxDbgSteps) ? dbg.p : nullptr;
            HIP_TRY(h, launch_dx(a, st));
        }
    }
    if (dbg.p) return dump_wave_stamps(h, dbg, dbg_n, kXcds * kXcdWgs * kDxWaves, dbg_steps, kDxStamps, st);
    return WRNN_OK;
}

int generate_dm(wrnn_t *h, int B, int L, const float *noise, uint64_t seed, int64_t row_offset, float *out,
                int32_t *labels, hipStream_t st) {
    // two row groups per launch (G/2 workgroups each) unless WRNN_ROW_GROUPS=1 or one row
    const char *gran_env = std::getenv("WRNN_ROWS_GRANULES");
    const int gran_force = gran_env ? std::atoi(gran_env) : -1;
    const char *grp_env = std::getenv("WRNN_ROW_GROUPS");
    const bool grouped = h->dm2.ok && B >= 2 && !(grp_env && std::atoi(grp_env) == 1);
    DmScope sc(*h, h->dm2, grouped);
    const int ng = grouped ? 2 : 1;
    const int S = h->cfg.rnn_dims / 2, Q = h->cfg.n_classes;
    const size_t flag_words = (size_t)kDmHops * kFlagSlots * kFlagStride, xg_words = (size_t)2 * kXReps * kXRepStride;
    for (int b0 = 0; b0 < B;) {
        int Bl = std::min(B - b0, kRowsMax);
        auto group_rows = [&](int bl, int g) { const int b_0 = (bl + ng - 1) / ng; return g == 0 ? b_0 : bl - b_0; };
        while (Bl > 1 && dm_tile_for(*h, group_rows(Bl, 0)) == 0) --Bl;
        const int Bg = group_rows(Bl, 0);
        const int TB = dm_tile_for(*h, Bg);
        if (TB == 0) return fail(h, WRNN_EUNSUPPORTED, "DM: one row of state does not fit LDS");
        const int SW = dm_state_width(h->dmU);
        const size_t act_grp = (size_t)kDmHops * 2 * Bg * h->KA, state_grp = (size_t)h->G * Bg * SW + 2 * Bg;
        if (grow(h, h->d_act, h->act_cap, ng * act_grp) || grow(h, h->d_state, h->state_cap, ng * state_grp))
            return WRNN_EHIP;
        HIP_TRY(h, ensure(h->d_dmflags, h->dmflags_cap, 2 * flag_words));
        HIP_TRY(h, ensure(h->d_dmxg, h->dmxg_cap, 2 * xg_words));
        HIP_TRY(h, hipMemsetAsync(h->d_dmflags, 0, ng * flag_words * 4, st));
        HIP_TRY(h, hipMemsetAsync(h->d_dmxg, 0, ng * xg_words * 8, st));
        // granule hand-offs while a group's hop vector is small (kDmGranMax values);
        // WRNN_ROWS_GRANULES=0|1 forces bulk / granules
        const bool gran = gran_force == 1 || (gran_force != 0 && (size_t)Bg * h->KA <= kDmGranMax);
        const long long gstride = (((long long)Bg * h->KA + kDmGranPad + 15) / 16) * 16;
        if (gran) {
            HIP_TRY(h, ensure(h->d_gact, h->gact_cap, (size_t)ng * kDmHops * gstride));
            HIP_TRY(h, hipMemsetAsync(h->d_gact, 0, (size_t)ng * kDmHops * gstride * 8, st));
        }
        DmArgs a{};
        a.slab = h->d_dmslab;
        a.noise = noise;
        a.out = out;
        a.labels = labels;
        a.act = h->d_act;
        a.flags = h->d_dmflags;
        a.xg = h->d_dmxg;
        a.gact = gran ? h->d_gact : nullptr;
        a.gstride = gstride;
        a.state = h->d_state;
        a.ctl = h->d_ctl;
        a.seed = seed;
        a.row0 = row_offset + b0;
        a.timeout_ticks = h->timeout_ticks;
        a.L = L;
        a.t0 = 0;
        a.Lc = L;
        a.B = Bg;
        a.Bt = B;
        a.b0 = b0;
        a.H = 2 * S;
        a.S = S;
        a.Q = Q;
        a.U = h->dmU;
        a.UO = h->dmUO;
        a.UO2 = h->dmUO2;
        a.G = h->G;
        a.TB = TB;
        a.KA = h->KA;
        a.s = h->ds;
        a.gw = h->dm_gw ? 1 : 0;
        DmGroup g1{};
        if (grouped) {
            g1.act = h->d_act + act_grp;
            g1.flags = h->d_dmflags + flag_words;
            g1.xg = h->d_dmxg + xg_words;
            g1.gact = gran ? h->d_gact + (size_t)kDmHops * gstride : nullptr;
            g1.state = h->d_state + state_grp;
            g1.row0 = row_offset + b0 + Bg;
            g1.B = group_rows(Bl, 1);
            g1.b0 = b0 + Bg;
        }
        HIP_TRY(h, launch_dm(a, grouped ? &g1 : nullptr, dm_lds_bytes(*h, Bg, TB), st));
        b0 += Bl;
    }
    return WRNN_OK;
}

// One MoL row through the role-split kernel: time chunks sized so terms + GEMM input stay within
// WRNN_TERMS_MB (default 8192 MiB).  Each chunk's terms cover one step past its end (step t's
// launch publishes the GRU1 terms of t + 1); the recurrent state is carried in d_state.
int generate_split(wrnn_t *h, const float *cond, int B, int L, const float *noise, uint64_t seed,
                   int64_t row_offset, float *out, hipStream_t st) {
    const wrnn_config &c = h->cfg;
    const int R = c.rnn_dims, A = c.aux_dims, G = h->sGg + h->sGf, N = G * kSplitTerms;
    if (!h->blas && rocblas_create_handle(&h->blas) != rocblas_status_success)
        return fail(h, WRNN_EHIP, "rocblas_create_handle failed");
    if (rocblas_set_stream(h->blas, st) != rocblas_status_success) return fail(h, WRNN_EHIP, "rocblas_set_stream failed");
    const char *mb_env = std::getenv("WRNN_TERMS_MB");
    const double budget = (mb_env ? std::atof(mb_env) : 8192.0) * (1 << 20) / 4.0;   // floats
    const int Lc_max = (int)std::max(1.0, std::min((double)L, budget / (double)(N + h->KX) - 1.0));
    const char *rep_env = std::getenv("WRNN_REPLICAS");
    // 4 replicas of every hand-off vector (profiles/r02_split_rep_sweep.log, two rounds): 5.73/5.79 us/step
    // vs 5.71/5.80 at 8, 5.75/5.90 at 2, 6.1-6.3 at 3, 6 and 16, 7.2 at 32; every count parity-green
    const int reps = std::max(1, std::min(32, rep_env ? std::atoi(rep_env) : 4));
    const long long vec_max = std::max<long long>({(long long)kTermsPerUnit * R, (long long)R, (long long)c.fc_dims,
                                                   (long long)(R / kSplitUnits) * kYLine,
                                                   (long long)h->sGf * kSplitLogitLine});
    const long long rep_stride = (((vec_max + kOverRead) * 8 + 65535) / 65536) * 65536 / 8;
    const size_t need_xg = (size_t)kSplitHops * reps * rep_stride;
    HIP_TRY(h, ensure(h->d_xg, h->xg_cap, need_xg));
    if (grow(h, h->d_X, h->X_cap, (size_t)(Lc_max + 1) * h->KX) || grow(h, h->d_T, h->T_cap, (size_t)(Lc_max + 1) * N) ||
        grow(h, h->d_state, h->state_cap, (size_t)G * split_state_w(R)))
        return WRNN_EHIP;
    const char *dbg_env = std::getenv("WRNN_DEBUG_STAMPS");
    const int dbg_steps = dbg_env ? std::min(L, std::atoi(dbg_env)) : 0;
    DbgBuf dbg;
    if (dbg_steps > 0) {
        HIP_TRY(h, hipMalloc(&dbg.p, (size_t)G * dbg_steps * kStamps * 4));
        HIP_TRY(h, hipMemsetAsync(dbg.p, 0, (size_t)G * dbg_steps * kStamps * 4, st));
    }
    const float one = 1.0f, zero = 0.0f;
    for (int b0 = 0; b0 < B; ++b0) {
        HIP_TRY(h, hipMemsetAsync(h->d_xg, 0, need_xg * 8, st));
        for (int t0 = 0; t0 < L; t0 += Lc_max) {
            const int Lc = std::min(Lc_max, L - t0);
            const int rows = std::min(Lc + 1, L - t0);     // terms rows: steps [t0, t0 + rows)
            HIP_TRY(h, launch_ci_gemm(cond, h->CD, B, b0, 1, t0, rows, h->d_IW, 1 + c.feat_dims + A, h->d_Ib, R,
                                      c.feat_dims + A, h->d_X, h->KX, st));
            HIP_TRY(h, launch_pack_terms_input(cond, h->CD, B, b0, 1, t0, rows, c.feat_dims, A, R, h->KX, h->d_X, st));
            if (rocblas_sgemm(h->blas, rocblas_operation_transpose, rocblas_operation_none, N, rows, h->KX, &one,
                              h->d_sWt, h->KX, h->d_X, h->KX, &zero, h->d_T, N) != rocblas_status_success)
                return fail(h, WRNN_EHIP, "rocblas_sgemm (conditioning terms) failed");
            SplitArgs a{};
            a.gslab = h->d_sgslab;
            a.fslab = h->d_sfslab;
            a.terms = h->d_T;
            a.noise = noise;
            a.out = out;
            a.state = h->d_state;
            a.xg = h->d_xg;
            a.ctl = h->d_ctl;
            a.seed = seed;
            a.row0 = row_offset + b0;
            a.timeout_ticks = h->timeout_ticks;
            a.rep_stride = rep_stride;
            a.L = L;
            a.t0 = t0;
            a.Lc = Lc;
            a.Bt = B;
            a.b0 = b0;
            a.Gg = h->sGg;
            a.Gf = h->sGf;
            a.reps = reps;
            a.gs = h->sgs;
            a.fs = h->sfs;
            a.dbg = (b0 == 0 && t0 == 0) ? dbg.p : nullptr;
            a.dbg_steps = std::min(dbg_steps, Lc);
            HIP_TRY(h, launch_split(a, split_lds_bytes(*h), st));
        }
    }
    if (dbg.p) return dump_stamps(h, dbg.release(), dbg_steps, st, G);
    return WRNN_OK;
}

// ---- frame-rate conditioning terms (frame_terms.hip) -------------------------------------
// A loop row's terms come from its utterance's frame rows: row r is utterance r / nf starting at
// step (r % nf)·stride (fold_with_overlap, fatchord_version.py:317-330; unbatched nf = 1).
struct FrameSrc {
    const float *mel = nullptr, *aux = nullptr;   // [U][feat][NF], [U][4·aux][NF] (device)
    int U = 0, NF = 0, nf = 1, stride = 0;
    int rb = 0;                                   // launch row j is row rb + j of the U·nf (wrnn_generate_frames_rows)
    int hop = 1, nJ = 1, jlo = 0;
    const float *coef = nullptr;                  // [hop][nJ] (device)
};

// The UpsampleNetwork's frame weights (fatchord_version.py:64-89): the response κ of pad →
// Stretch2d(s_i) → Conv2d(1, 2s_i+1, pad s_i) (×n) to one unit frame, in float64, as
// coef[φ][k] = κ(φ − hop·(k + jlo)).  Each stage spreads a frame by ±s_i samples at its rate,
// E = Σ s_i·hop / r_i samples at the output rate (r_i = s_1···s_i): κ lives on [−E, hop − 1 + E].
// Exact (equal to the stage-wise zero-padded cascade over the cropped output) when the pad
// frames cover that reach: pad·hop ≥ E.  Returns false otherwise (the caller keeps the
// per-sample conditioning path).
bool frame_weights(const wrnn_upsample_cfg &c, int *hop_out, int *nJ_out, int *jlo_out, std::vector<float> &coef) {
    int hop = 1;
    for (int i = 0; i < c.n_scales; ++i) hop *= c.scales[i];
    long long E = 0;
    for (int i = 0, r = 1; i < c.n_scales; ++i) {
        r *= c.scales[i];
        E += (long long)c.scales[i] * (hop / r);
    }
    if ((long long)c.pad * hop < E) return false;
    const int jlo = -(int)((hop - 1 + E) / hop), jhi = (int)((E + hop - 1) / hop);
    const int nJ = jhi - jlo + 1;
    if (nJ > 8) return false;
    // unit frame at index W of 2W + 1 frames, W beyond the reach
    const int W = jhi - jlo + 1;
    std::vector<double> x(2 * W + 1, 0.0);
    x[W] = 1.0;
    for (int i = 0; i < c.n_scales; ++i) {
        const int s = c.scales[i];
        std::vector<double> y(x.size() * s), z(x.size() * s, 0.0);
        for (size_t n = 0; n < y.size(); ++n) y[n] = x[n / s];
        for (long long n = 0; n < (long long)z.size(); ++n) {
            double acc = 0.0;
            for (int m = 0; m <= 2 * s; ++m) {
                const long long q = n + m - s;
                if (q >= 0 && q < (long long)y.size()) acc += (double)c.taps[i][m] * y[q];
            }
            z[n] = acc;
        }
        x.swap(z);
    }
    coef.assign((size_t)hop * nJ, 0.0f);
    for (int ph = 0; ph < hop; ++ph)
        for (int k = 0; k < nJ; ++k) {
            const long long d = ph - (long long)hop * (k + jlo);   // output offset from the frame's first sample
            const long long n = d + (long long)W * hop;
            if (n >= 0 && n < (long long)x.size()) coef[(size_t)ph * nJ + k] = (float)x[n];
        }
    *hop_out = hop;
    *nJ_out = nJ;
    *jlo_out = jlo;
    return true;
}

// FT [NF + nJ − 1][U][N] = W·[mel frame | 0 | 0] and AT [NF + 1][U][N] = W·[0 | aux frame | 1]
// (row NF: W·[0 | 0 | 1]) through the path's own terms GEMM(s): gemm(X, m, C) writes
// C[m][N] = W·X for X [m][KX] as pack_cond_input lays it out (`split`).
template <typename Gemm>
int frame_terms(wrnn_t *h, const FrameSrc &fs, int N, int KX, int split, hipStream_t st, Gemm gemm) {
    const int feat = h->cfg.feat_dims, A4 = h->CD - feat;
    const int NFF = fs.NF + fs.nJ - 1, NFA = fs.NF + 1, fmax = std::max(NFF, NFA);
    if (grow(h, h->d_frec, h->frec_cap, (size_t)fmax * fs.U * h->CD) ||
        grow(h, h->d_X, h->X_cap, (size_t)fmax * fs.U * KX) || grow(h, h->d_FT, h->FT_cap, (size_t)NFF * fs.U * N) ||
        grow(h, h->d_AT, h->AT_cap, (size_t)NFA * fs.U * N))
        return WRNN_EHIP;
    for (int kind = 0; kind < 2; ++kind) {
        const int frames = kind ? NFA : NFF;
        HIP_TRY(h, launch_frame_cond(fs.mel, fs.aux, fs.U, feat, A4, fs.NF, frames, fs.jlo, kind, h->d_frec, st));
        HIP_TRY(h, launch_pack_cond_input(h->d_frec, h->CD, fs.U, 0, fs.U, 0, frames, KX, h->d_X, st, split,
                                          kind ? 1.0f : 0.0f));
        if (int rc = gemm(h->d_X, frames * fs.U, kind ? h->d_AT : h->d_FT)) return rc;
    }
    return WRNN_OK;
}

// MoL rows through the XCD-resident kernel: up to 8 rows per launch (row k on XCD k), time
// chunks sized so terms + GEMM input stay within WRNN_TERMS_MB (default 8192 MiB).  Each chunk's
// terms cover one step past its end (step t publishes the GRU1 terms of t + 1); the recurrent
// state is carried per workgroup in d_xstate.
// The one-row-per-XCD kernels (fatchord_xcd: dense rnn 512, fatchord_xcds: block-sparse rnn 896)
// share this launch loop: rows in groups of 8 (one per XCD), time chunks whose precomputed terms
// fit the WRNN_TERMS_MB budget, one terms GEMM per chunk (one step ahead: the kernels prefetch
// the terms of step t + 1), the recurrent state carried per workgroup between chunks.
// n_terms = terms per workgroup and step, state_w = carried floats per workgroup.
template <typename Args, typename Slab>
int generate_xcd_rows(wrnn_t *h, const float *cond, const FrameSrc *fs, int B, int L, const float *noise,
                      uint64_t seed, int64_t row_offset, float *out, hipStream_t st, int n_terms, int state_w,
                      const Slab &slab, hipError_t (*launch)(const Args &, hipStream_t)) {
    const int N = kXcdWgs * n_terms;
    if (!h->blas && rocblas_create_handle(&h->blas) != rocblas_status_success)
        return fail(h, WRNN_EHIP, "rocblas_create_handle failed");
    if (rocblas_set_stream(h->blas, st) != rocblas_status_success) return fail(h, WRNN_EHIP, "rocblas_set_stream failed");
    if (fs) {   // frame-rate terms: W·(frames) once, then per chunk the nJ-tap sum (frame_terms.hip)
        const float one = 1.0f, zero = 0.0f;
        const int rc = frame_terms(h, *fs, N, h->KXc, 0, st, [&](const float *X, int m, float *C) -> int {
            if (rocblas_sgemm(h->blas, rocblas_operation_transpose, rocblas_operation_none, N, m, h->KXc, &one,
                              h->d_xWt, h->KXc, X, h->KXc, &zero, C, N) != rocblas_status_success)
                return fail(h, WRNN_EHIP, "rocblas_sgemm (frame terms) failed");
            return WRNN_OK;
        });
        if (rc) return rc;
    }
    const char *mb_env = std::getenv("WRNN_TERMS_MB");
    const double budget = (mb_env ? std::atof(mb_env) : 8192.0) * (1 << 20) / 4.0;   // floats
    const size_t xg_words = (size_t)kXcds * kXXcdStride;
    // each buffer under its own check: generate_xcdm / generate_dx allocate d_members too
    if (!h->d_members) HIP_TRY(h, hipMalloc(&h->d_members, kXcds * sizeof(int)));
    if (!h->d_xgx) HIP_TRY(h, hipMalloc(&h->d_xgx, xg_words * 8));
    const char *dbg_env = std::getenv("WRNN_DEBUG_STAMPS");
    const int dbg_steps = dbg_env ? std::min(L, std::atoi(dbg_env)) : 0;
    DbgBuf dbg;
    int dbg_G = 0;
    const float one = 1.0f, zero = 0.0f;
    for (int b0 = 0; b0 < B; b0 += kXcds) {
        const int nb = std::min(kXcds, B - b0);
        const int Lc_max = (int)std::max(1.0, std::min((double)L, budget / ((double)nb * (N + h->KXc)) - 1.0));
        if (grow(h, h->d_X, h->X_cap, (size_t)(Lc_max + 1) * nb * h->KXc) ||
            grow(h, h->d_T, h->T_cap, (size_t)(Lc_max + 1) * nb * N) ||
            grow(h, h->d_xstate, h->xstate_cap, (size_t)nb * kXcdWgs * state_w))
            return WRNN_EHIP;
        if (dbg_steps > 0 && !dbg.p) {
            dbg_G = nb * kXcdWgs;
            HIP_TRY(h, hipMalloc(&dbg.p, (size_t)dbg_G * dbg_steps * kStamps * 4));
            HIP_TRY(h, hipMemsetAsync(dbg.p, 0, (size_t)dbg_G * dbg_steps * kStamps * 4, st));
        }
        HIP_TRY(h, hipMemsetAsync(h->d_xgx, 0, (size_t)nb * kXXcdStride * 8, st));   // tags restart at 1
        for (int t0 = 0; t0 < L; t0 += Lc_max) {
            const int Lc = std::min(Lc_max, L - t0);
            const int rows = std::min(Lc + 1, L - t0);     // terms rows: steps [t0, t0 + rows)
            if (fs) {
                HIP_TRY(h, launch_terms_interp(h->d_FT, h->d_AT, fs->coef, h->d_T, N, fs->U, fs->NF, fs->NF + fs->nJ - 1,
                                               fs->hop, fs->nJ, fs->nf, fs->stride, fs->rb + b0, nb, t0, rows, st));
            } else {
                HIP_TRY(h, launch_pack_cond_input(cond, h->CD, B, b0, nb, t0, rows, h->KXc, h->d_X, st));
                if (rocblas_sgemm(h->blas, rocblas_operation_transpose, rocblas_operation_none, N, rows * nb, h->KXc,
                                  &one, h->d_xWt, h->KXc, h->d_X, h->KXc, &zero, h->d_T, N) != rocblas_status_success)
                    return fail(h, WRNN_EHIP, "rocblas_sgemm (conditioning terms) failed");
            }
            HIP_TRY(h, hipMemsetAsync(h->d_members, 0, kXcds * sizeof(int), st));
            Args a{};
            a.slab = h->d_xslab;
            a.terms = h->d_T;
            a.noise = noise;
            a.out = out;
            a.state = h->d_xstate;
            a.xg = h->d_xgx;
            a.members = h->d_members;
            a.ctl = h->d_ctl;
            a.seed = seed;
            a.row0 = row_offset + b0;
            a.timeout_ticks = h->timeout_ticks;
            a.L = L;
            a.t0 = t0;
            a.Lc = Lc;
            a.Bt = B;
            a.b0 = b0;
            a.nb = nb;
            a.s = slab;
            a.dbg = (b0 == 0 && t0 == 0) ? dbg.p : nullptr;
            a.dbg_steps = std::min(dbg_steps, Lc);
            HIP_TRY(h, launch(a, st));
        }
    }
    if (dbg.p) return dump_stamps(h, dbg.release(), dbg_steps, st, dbg_G);
    return WRNN_OK;
}

int generate_xcd(wrnn_t *h, const float *cond, const FrameSrc *fs, int B, int L, const float *noise, uint64_t seed,
                 int64_t row_offset, float *out, hipStream_t st) {
    return generate_xcd_rows<XcdArgs>(h, cond, fs, B, L, noise, seed, row_offset, out, st, kXTerms, kXStateW, h->xs,
                                      launch_xcd);
}

int generate_xcds(wrnn_t *h, const float *cond, const FrameSrc *fs, int B, int L, const float *noise, uint64_t seed,
                  int64_t row_offset, float *out, hipStream_t st) {
    return generate_xcd_rows<XcdsArgs>(h, cond, fs, B, L, noise, seed, row_offset, out, st, kSTerms, kSStateW, h->xss,
                                       launch_xcds);
}

// MoL rows through the XCD-resident many-row kernel: up to kMRowsMax rows per launch (launch row
// r on XCD r % 8, its row r / 8 there), time chunks sized so terms + GEMM input stay within
// WRNN_TERMS_MB (default 8192 MiB); the recurrent state is carried per workgroup in d_xmstate.
int generate_xcdm(wrnn_t *h, const float *cond, const FrameSrc *fs, int B, int L, const float *noise, uint64_t seed,
                  int64_t row_offset, float *out, int32_t *labels, hipStream_t st) {
    const int N = kXcdWgs * kMRing;   // compact terms record (d_xmWt)
    const bool raw = h->cfg.mode == WRNN_MODE_RAW;
    const int NK = raw ? kMRawNC : 11;              // draws per row-step: Exp(1) per class / MoL uniforms
    if (!h->blas && rocblas_create_handle(&h->blas) != rocblas_status_success)
        return fail(h, WRNN_EHIP, "rocblas_create_handle failed");
    if (rocblas_set_stream(h->blas, st) != rocblas_status_success) return fail(h, WRNN_EHIP, "rocblas_set_stream failed");
    const char *mb_env = std::getenv("WRNN_TERMS_MB");
    const double budget = (mb_env ? std::atof(mb_env) : 8192.0) * (1 << 20) / 4.0;   // floats
    const size_t xg_words = (size_t)kXcds * kMXcdStride;
    if (!h->d_members) HIP_TRY(h, hipMalloc(&h->d_members, kXcds * sizeof(int)));
    if (!h->d_xmxg) HIP_TRY(h, hipMalloc(&h->d_xmxg, xg_words * 8));
    if (!h->d_xmstate) HIP_TRY(h, hipMalloc(&h->d_xmstate, (size_t)kXcds * kXcdWgs * kMStateW * sizeof(float)));
    const int rows_max = kXcds * 4 * h->xcdm_nq;
    const float one = 1.0f, zero = 0.0f;
    XcdmGemm gemms[3];
    xcdm_terms_gemms(*h, gemms);
    // the segmented terms GEMMs writing C[m][N] for X [m][KXc]
    auto terms_gemm = [&](const float *X, int m, float *C) -> int {
        for (const XcdmGemm &g : gemms) {
            const rocblas_status rs =
                rocblas_sgemm(h->blas, rocblas_operation_transpose, rocblas_operation_none, g.rows, m, g.k, &one,
                              h->d_xmWt + (size_t)g.row0 * h->KXc + g.col0, h->KXc, X + g.col0, h->KXc, &zero,
                              C + g.row0, N);
            if (rs != rocblas_status_success) return fail(h, WRNN_EHIP, "rocblas_sgemm (conditioning terms) failed");
        }
        return WRNN_OK;
    };
    if (fs) {   // frame-rate terms (frame_terms.hip)
        if (int rc = frame_terms(h, *fs, N, h->KXc, h->cfg.feat_dims + h->cfg.aux_dims, st, terms_gemm)) return rc;
    }
    // diagnostics: WRNN_DEBUG_STAMPS=1 WRNN_DEBUG_FILE=<path>: per-wave phase stamps of the first
    // launch ([256 · kMWaves][kMDbgSteps][kMStamps] shader clocks, int32 header)
    const char *dbg_env = std::getenv("WRNN_DEBUG_STAMPS");
    const int dbg_steps = (!raw && dbg_env && std::atoi(dbg_env) > 0 && L >= kMDbgSkip + kMDbgSteps) ? kMDbgSteps : 0;
    const size_t dbg_n = (size_t)kXcds * kXcdWgs * kMWaves * dbg_steps * kMStamps;
    DbgBuf dbg;
    if (dbg_steps > 0) {
        HIP_TRY(h, hipMalloc(&dbg.p, dbg_n * 4));
        HIP_TRY(h, hipMemsetAsync(dbg.p, 0, dbg_n * 4, st));
    }
    for (int b0 = 0; b0 < B; b0 += rows_max) {
        const int nb = std::min(rows_max, B - b0);
        const int nq = (((nb + kXcds - 1) / kXcds) + 3) / 4;   // quads on the fullest XCD
        const int Lc_max = (int)std::max(1.0, std::min((double)L, budget / ((double)nb * (N + h->KXc + (noise ? 0 : NK)))));
        if (grow(h, h->d_X, h->X_cap, (size_t)Lc_max * nb * h->KXc) || grow(h, h->d_T, h->T_cap, (size_t)Lc_max * nb * N) ||
            (!noise && grow(h, h->d_xmnoise, h->xmnoise_cap, (size_t)Lc_max * nb * NK)))
            return WRNN_EHIP;
        // tags restart at 1, every packed hop element empty (fatchord_xcdm.h: all bits set)
        HIP_TRY(h, hipMemsetAsync(h->d_xmxg, 0xFF, xg_words * 8, st));
        for (int t0 = 0; t0 < L; t0 += Lc_max) {
            const int Lc = std::min(Lc_max, L - t0);
            if ((size_t)Lc * nb * h->KXc > h->X_cap || (size_t)Lc * nb * N > h->T_cap)
                return fail(h, WRNN_EINVAL, "xcdm: terms workspace too small");
            if (fs) {
                HIP_TRY(h, launch_terms_interp(h->d_FT, h->d_AT, fs->coef, h->d_T, N, fs->U, fs->NF, fs->NF + fs->nJ - 1,
                                               fs->hop, fs->nJ, fs->nf, fs->stride, fs->rb + b0, nb, t0, Lc, st));
            } else {
                HIP_TRY(h, launch_pack_cond_input(cond, h->CD, B, b0, nb, t0, Lc, h->KXc, h->d_X, st,
                                                  h->cfg.feat_dims + h->cfg.aux_dims));
                if (int rc = terms_gemm(h->d_X, Lc * nb, h->d_T)) return rc;
            }
            HIP_TRY(h, hipMemsetAsync(h->d_members, 0, kXcds * sizeof(int), st));
            XcdmArgs a{};
            a.slab = h->d_xmslab;
            a.terms = h->d_T;
            if (noise) {   // injected [L][B][NK]
                a.noise = noise;
                a.nz_t0 = 0;
                a.nz_ts = B;
                a.nz_b0 = b0;
            } else {       // Philox, drawn for this chunk by a small kernel first ([Lc][nb][NK])
                HIP_TRY(h, launch_philox_fill(h->d_xmnoise, seed, row_offset + b0, nb, t0, Lc, NK, raw ? 0 : 1, st));
                a.noise = h->d_xmnoise;
                a.nz_t0 = t0;
                a.nz_ts = nb;
                a.nz_b0 = 0;
            }
            a.out = out;
            a.labels = labels;
            a.state = h->d_xmstate;
            a.xg = h->d_xmxg;
            a.members = h->d_members;
            a.ctl = h->d_ctl;
            a.seed = seed;
            a.row0 = row_offset + b0;
            a.timeout_ticks = h->timeout_ticks;
            a.L = L;
            a.t0 = t0;
            a.Lc = Lc;
            a.Bt = B;
            a.b0 = b0;
            a.nb = nb;
            a.s = h->xms;
            a.dbg = (b0 == 0 && t0 == 0 && Lc >= kMDbgSkip + kMDbgSteps) ? dbg.p : nullptr;
            HIP_TRY(h, launch_xcdm(a, nq, raw, st));
        }
    }
    if (dbg.p) return dump_wave_stamps(h, dbg, dbg_n, kXcds * kXcdWgs * kMWaves, dbg_steps, kMStamps, st);
    return WRNN_OK;
}

int generate_latency(wrnn_t *h, const float *cond, int B, int L, const float *noise, uint64_t seed,
                     int64_t row_offset, float *out, int32_t *labels, hipStream_t st) {
    const wrnn_config &c = h->cfg;
    const int R = c.rnn_dims;
    const int Bc_max = std::min(B, h->max_rows);
    // workspaces (grow-only)
    if (grow(h, h->d_cI, h->cI_cap, (size_t)L * Bc_max * R)) return WRNN_EHIP;
    // hand-off replicas (WRNN_REPLICAS, default 8), each padded to a 64 KiB boundary; at most
    // 64 / kTermsPerUnit, since one wave publishes every term of a unit to every replica at once
    // (8 measured best: 8.18 us/step at rnn 512 B=1; 4 -> 8.27, 16 -> 8.77, 2 -> 8.84)
    const char *rep_env = std::getenv("WRNN_REPLICAS");
    const int reps = std::max(1, std::min(64 / kTermsPerUnit, rep_env ? std::atoi(rep_env) : 8));
    // replica stride ≥ 64 KiB: keeps replicas on different lines/channels and makes the
    // pollers' fixed-count over-reads (slots ≥ n) land in allocated memory
    const long long vec_max = std::max<long long>({(long long)Bc_max * h->NMAX, (long long)Bc_max * R * kTermsPerUnit,
                                                   3LL * R});
    const long long rep_stride = (((vec_max + kOverRead) * 8 + 65535) / 65536) * 65536 / 8;
    const size_t need_xg = (size_t)kHops * reps * rep_stride;
    HIP_TRY(h, ensure(h->d_xg, h->xg_cap, need_xg));
    // diagnostics: WRNN_DEBUG_STAMPS=<steps> WRNN_DEBUG_FILE=<path> dumps per-stage stamps
    const char *dbg_env = std::getenv("WRNN_DEBUG_STAMPS");
    const int dbg_steps = dbg_env ? std::min(L, std::atoi(dbg_env)) : 0;
    DbgBuf dbg;
    if (dbg_steps > 0) {
        HIP_TRY(h, hipMalloc(&dbg.p, (size_t)h->G * dbg_steps * kStamps * 4));
        HIP_TRY(h, hipMemsetAsync(dbg.p, 0, (size_t)h->G * dbg_steps * kStamps * 4, st));
    }
    for (int b0 = 0; b0 < B; b0 += h->max_rows) {
        const int Bc = std::min(h->max_rows, B - b0);
        HIP_TRY(h, launch_ci_gemm(cond, h->CD, B, b0, Bc, 0, L, h->d_IW, 1 + c.feat_dims + c.aux_dims, h->d_Ib, R,
                                  c.feat_dims + c.aux_dims, h->d_cI, R, st));
        HIP_TRY(h, hipMemsetAsync(h->d_xg, 0, need_xg * 8, st));
        LoopArgs a{};
        a.slab = h->d_slab;
        a.cI = h->d_cI;
        a.cond = cond;
        a.noise = noise;
        a.out = out;
        a.labels = labels;
        a.xg = h->d_xg;
        a.reps = reps;
        {
            const char *dp = std::getenv("WRNN_DELAY_POLL");
            a.delay_poll = dp ? std::atoi(dp) : 1;
        }
        a.rep_stride = rep_stride;
        a.ctl = h->d_ctl;
        a.seed = seed;
        a.row0 = row_offset + b0;
        a.timeout_ticks = h->timeout_ticks;
        a.L = L;
        a.Bc = Bc;
        a.Bt = B;
        a.b0 = b0;
        a.R = R;
        a.F = c.fc_dims;
        a.A = c.aux_dims;
        a.CD = h->CD;
        a.feat = c.feat_dims;
        a.NC = c.n_classes;
        a.NK = h->NK;
        a.mol = c.mode == WRNN_MODE_MOL;
        a.U = h->U;
        a.UF = h->UF;
        a.UC = h->UC;
        a.G = h->G;
        a.NMAX = h->NMAX;
        a.s = h->s;
        a.dbg = (b0 == 0) ? dbg.p : nullptr;
        a.dbg_steps = dbg_steps;
        HIP_TRY(h, launch_loop(a, lds_bytes_for(*h, Bc), st));
    }
    if (dbg.p) return dump_stamps(h, dbg.release(), dbg_steps, st, h->G);
    return WRNN_OK;
}

}  // namespace

extern "C" {

int wrnn_create(const wrnn_config *cfg, int device, wrnn_t **out) {
    if (!out || !cfg) return WRNN_EINVAL;
    *out = nullptr;
    if (cfg->abi_version != WRNN_ABI_VERSION) return WRNN_EINVAL;
    auto *h = new (std::nothrow) wrnn_ctx();
    if (!h) return WRNN_ENOMEM;
    *out = h;
    h->cfg = *cfg;
    h->device = device;
    const wrnn_config &c = h->cfg;
    const bool mol = c.mode == WRNN_MODE_MOL;
    if (c.mode != WRNN_MODE_MOL && c.mode != WRNN_MODE_RAW && c.mode != WRNN_MODE_DM)
        return fail(h, WRNN_EINVAL, "unknown mode");
    if (c.rnn_dims <= 0 || c.n_classes <= 0 ||
        (c.mode != WRNN_MODE_DM && (c.fc_dims <= 0 || c.aux_dims <= 0 || c.feat_dims <= 0)))
        return fail(h, WRNN_EINVAL, "dims must be positive");
    if (c.mode != WRNN_MODE_DM && (c.rnn_dims % 4 || c.fc_dims % 4 || c.aux_dims % 4))
        return fail(h, WRNN_EUNSUPPORTED, "rnn_dims, fc_dims and aux_dims must be multiples of 4");
    if (mol && c.n_classes != 30) return fail(h, WRNN_EINVAL, "MOL mode has n_classes = 30 (10 logistics)");
    HIP_TRY(h, hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(h, hipGetDeviceProperties(&prop, device));
    h->num_cus = prop.multiProcessorCount;
    h->max_lds = std::max<int>((int)prop.sharedMemPerBlock, (int)prop.maxSharedMemoryPerMultiProcessor);
    h->max_lds = std::min(h->max_lds, 160 * 1024);
    if (c.mode == WRNN_MODE_DM) {   // deepmind_version: the multi-row dual-softmax kernel only
        const int H = c.rnn_dims, S = H / 2, Q = c.n_classes;
        if (S % 4) return fail(h, WRNN_EUNSUPPORTED, "DM hidden_size must be a multiple of 8");
        const int gt = c.grid > 0 ? c.grid : h->num_cus;
        h->dm = true;
        h->dmU = (S + gt - 1) / gt;
        h->G = (S + h->dmU - 1) / h->dmU;
        h->dmUO = (S + h->G - 1) / h->G;
        h->dmUO2 = (Q + h->G - 1) / h->G;
        h->KA = round4(std::max(S, Q));
        h->NK = 2 * Q;
        h->ds = make_dm_slab(*h);
        if (dm_tile_for(*h, 1) == 0) h->dm_gw = true;   // weights beyond LDS: stream the slab
        if (dm_tile_for(*h, 1) == 0)
            return fail(h, WRNN_EUNSUPPORTED, "DM: one row of state does not fit LDS (" + std::to_string(dm_lds_bytes(*h, 1, 1)) + " B)");
        HIP_TRY(h, prepare_dm_kernel(h->max_lds));
        int per_cu = 0;
        HIP_TRY(h, dm_occupancy(&per_cu, dm_lds_bytes(*h, 1, 1)));
        if (per_cu * h->num_cus < h->G)
            return fail(h, WRNN_EUNSUPPORTED, "DM persistent grid is not co-resident");
        // two row groups of G/2 workgroups (twice the units each), as the fatchord rows kernel
        if (h->G % 2 == 0 && h->G >= 8 && !h->dm_gw) {
            DmPart p{};
            p.G = h->G / 2;
            p.dmU = (S + p.G - 1) / p.G;
            p.G = (S + p.dmU - 1) / p.dmU;
            p.dmUO = (S + p.G - 1) / p.G;
            p.dmUO2 = (Q + p.G - 1) / p.G;
            h->dm2 = p;
            bool ok = false;
            {
                DmScope sc(*h, h->dm2, true);
                h->ds = make_dm_slab(*h);
                if (dm_tile_for(*h, 2) > 0) {
                    HIP_TRY(h, dm_occupancy(&per_cu, dm_lds_bytes(*h, 1, 1)));
                    ok = per_cu * h->num_cus >= 2 * h->G;
                }
            }
            h->dm2.ok = ok;
        }
        // hidden 896 / quantisation 256 on a full 8 × 32-CU MI355X: the XCD-resident MFMA kernel
        if (H == kDxH && Q == kDxQ && c.grid <= 0 && h->num_cus == kXcds * kXcdWgs) {
            bool ok = false;
            HIP_TRY(h, prepare_dx_kernel(h->max_lds, &ok));
            h->dx_ok = ok;
        }
        h->timeout_ticks = (long long)(c.timeout_ms > 0 ? c.timeout_ms : 2000) * 100000LL;
        HIP_TRY(h, hipMalloc(&h->d_ctl, kCtlWords * sizeof(int)));
        HIP_TRY(h, hipMemset(h->d_ctl, 0, kCtlWords * sizeof(int)));
        HIP_TRY(h, hipEventCreate(&h->ev0));
        HIP_TRY(h, hipEventCreate(&h->ev1));
        return WRNN_OK;
    }
    const int R = c.rnn_dims, F = c.fc_dims;
    const int gtarget = c.grid > 0 ? c.grid : h->num_cus;
    h->U = (R + gtarget - 1) / gtarget;
    h->G = (R + h->U - 1) / h->U;
    h->UF = (F + h->G - 1) / h->G;
    h->UC = mol ? 0 : (c.n_classes + h->G - 1) / h->G;
    h->NMAX = std::max(R, std::max(F, c.n_classes));
    h->NK = mol ? 11 : c.n_classes;
    h->CD = c.feat_dims + 4 * c.aux_dims;
    h->s = make_slab_layout(*h);
    // rows per launch: LDS, and the per-thread gather register budget
    h->KX = R + 3 * c.aux_dims + 4;
    h->KXc = h->CD + 4;
    h->KA = round4(std::max(R, std::max(F, c.n_classes)));
    set_rows_partition(*h, 0);
    // dims whose dense weights fit neither kernel may still run with block-sparse GRU weights
    // (decided at wrnn_set_weights)
    const bool sparse_possible = R % 4 == 0 && R / 4 <= h->num_cus;
    h->max_rows = 0;
    for (int b = 1; b <= 64; ++b) {
        if (lds_bytes_for(*h, b) > (size_t)h->max_lds) break;
        // one polling wave: kGatherMax slots per lane in the generic kernels, exact counts (rows ≤ 2)
        // in the compile-time-dims ones
        const bool fast = loop_has_fast_path(R, F, c.aux_dims, c.n_classes, mol, h->U, h->UF, h->UC);
        if (fast ? b > 2 : (size_t)b * h->NMAX > (size_t)kPollThreads * kGatherMax) break;
        h->max_rows = b;
    }
    if (h->max_rows < 1 && !h->rows_ok && !sparse_possible)
        return fail(h, WRNN_EUNSUPPORTED, "weight slab + one row of state exceeds LDS (" +
                                              std::to_string(lds_bytes_for(*h, 1)) + " B)");
    HIP_TRY(h, prepare_loop_kernel(h->max_lds));
    HIP_TRY(h, prepare_rows_kernel(h->max_lds));
    int per_cu = 0;
    if (h->max_rows >= 1) {
        HIP_TRY(h, loop_occupancy(&per_cu, lds_bytes_for(*h, h->max_rows)));
        if (per_cu * h->num_cus < h->G)
            return fail(h, WRNN_EUNSUPPORTED, "persistent grid of " + std::to_string(h->G) +
                                                  " workgroups is not co-resident (" + std::to_string(per_cu) +
                                                  "/CU × " + std::to_string(h->num_cus) + " CUs)");
    }
    if (h->rows_ok) {
        HIP_TRY(h, rows_occupancy(&per_cu, rows_lds_bytes(*h, 1, 1)));
        if (per_cu * h->num_cus < h->rG) h->rows_ok = false;
    }
    set_group_partition(*h);
    if (h->g2.ok) {
        PartScope ps(*h, h->g2, true);
        HIP_TRY(h, rows_occupancy(&per_cu, rows_lds_bytes(*h, 1, 1)));
        if (per_cu * h->num_cus < 2 * h->rG) h->rows_ok = false;
    }
    // one MoL row: the role-split kernel (compile-time dims) when its grid and LDS fit; an
    // explicit grid request keeps the uniform kernels
    if (mol && c.grid <= 0 && split_has_kernel(R, F) && R % kSplitUnits == 0 && F % kSplitFcRows == 0) {
        h->sGg = R / kSplitUnits;
        h->sGf = F / kSplitFcRows;
        make_split_slabs(*h);
        if (h->sGg + h->sGf <= h->num_cus && split_lds_bytes(*h) <= (size_t)h->max_lds) {
            HIP_TRY(h, prepare_split_kernel(h->max_lds));
            HIP_TRY(h, split_occupancy(&per_cu, split_lds_bytes(*h)));
            h->split_ok = per_cu >= 1;
        }
    }
    // MoL rnn / fc 512: the XCD-resident kernel (one row per XCD) on a full 8 × 32-CU MI355X
    if (mol && c.grid <= 0 && R == 512 && F == 512 && c.aux_dims == 32 && h->num_cus == kXcds * kXcdWgs &&
        xcd_lds_layout().total * sizeof(float) <= (size_t)h->max_lds) {
        make_xcd_slab(*h);
        HIP_TRY(h, prepare_xcd_kernel(h->max_lds));
        HIP_TRY(h, xcd_occupancy(&per_cu));
        h->xcd_ok = per_cu >= 1;
        // its many-row form (same terms GEMM)
        if (h->xcd_ok) {
            make_xcdm_slab(*h);
            HIP_TRY(h, prepare_xcdm_kernel(h->max_lds));
            HIP_TRY(h, xcdm_max_quads(h->max_lds, false, &h->xcdm_nq));
            h->xcdm_ok = h->xcdm_nq >= 1;
        }
    }
    // RAW 9-bit, rnn / fc 512: the many-row XCD-resident kernel with the softmax head (every row count)
    if (!mol && c.grid <= 0 && R == 512 && F == 512 && c.aux_dims == 32 && c.n_classes == kMRawNC &&
        h->num_cus == kXcds * kXcdWgs) {
        make_xcdm_slab(*h);
        HIP_TRY(h, prepare_xcdm_kernel(h->max_lds));
        HIP_TRY(h, xcdm_max_quads(h->max_lds, true, &h->xcdm_nq));
        h->xcdm_ok = h->xcdm_nq >= 1;
    }
    // MoL rnn 896 / fc 512: the XCD-resident block-sparse kernel, if the weights turn out
    // block-sparse (decided at wrnn_set_weights)
    if (mol && c.grid <= 0 && R == kSR && F == 512 && c.aux_dims == 32 && h->num_cus == kXcds * kXcdWgs &&
        xcds_lds_layout().total * sizeof(float) <= (size_t)h->max_lds) {
        make_xcds_slab(*h);
        HIP_TRY(h, prepare_xcds_kernel(h->max_lds));
        HIP_TRY(h, xcds_occupancy(&per_cu));
        h->xcds_cap = per_cu >= 1;
    }
    h->timeout_ticks = (long long)(c.timeout_ms > 0 ? c.timeout_ms : 2000) * 100000LL;   // 100 MHz
    HIP_TRY(h, hipMalloc(&h->d_ctl, kCtlWords * sizeof(int)));
    HIP_TRY(h, hipMemset(h->d_ctl, 0, kCtlWords * sizeof(int)));
    HIP_TRY(h, hipEventCreate(&h->ev0));
    HIP_TRY(h, hipEventCreate(&h->ev1));
    return WRNN_OK;
}

int wrnn_set_weights(wrnn_t *h, const wrnn_tensor *tensors, int n) {
    if (!h || (n > 0 && !tensors)) return WRNN_EINVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    const auto need = required(h->cfg);
    for (int i = 0; i < n; ++i) {
        const wrnn_tensor &t = tensors[i];
        if (!t.name || !t.data) return fail(h, WRNN_EINVAL, "null tensor name/data");
        auto it = std::find_if(need.begin(), need.end(), [&](const Need &q) { return t.name == std::string(q.name); });
        if (it == need.end()) continue;   // load_state_dict(strict=False): ignore others
        if (t.numel != it->rows * it->cols)
            return fail(h, WRNN_EINVAL, std::string(t.name) + ": expected " + std::to_string(it->rows * it->cols) +
                                            " elements, got " + std::to_string(t.numel));
        std::vector<float> v((size_t)t.numel);
        if (t.on_device)
            HIP_TRY(h, hipMemcpy(v.data(), t.data, (size_t)t.numel * 4, hipMemcpyDeviceToHost));
        else
            std::memcpy(v.data(), t.data, (size_t)t.numel * 4);
        h->w[t.name] = std::move(v);
    }
    for (const auto &q : need)
        if (!h->w.count(q.name)) { h->ready = false; return WRNN_OK; }   // partial load so far
    if (h->dm) {
        for (int grouped = 0; grouped < (h->dm2.ok ? 2 : 1); ++grouped) {
            DmScope sc(*h, h->dm2, grouped == 1);
            std::vector<float> slab((size_t)h->G * h->ds.total);
            for (int w = 0; w < h->G; ++w) pack_dm_slab(*h, w, slab.data() + (size_t)w * h->ds.total);
            if (h->d_dmslab) HIP_TRY(h, hipFree(h->d_dmslab));
            h->d_dmslab = nullptr;
            HIP_TRY(h, hipMalloc(&h->d_dmslab, slab.size() * 4));
            HIP_TRY(h, hipMemcpy(h->d_dmslab, slab.data(), slab.size() * 4, hipMemcpyHostToDevice));
        }
        if (h->dx_ok) {
            std::vector<float> slab;
            pack_dx_slab(*h, slab);
            if (h->d_dxslab) HIP_TRY(h, hipFree(h->d_dxslab));
            h->d_dxslab = nullptr;
            HIP_TRY(h, hipMalloc(&h->d_dxslab, slab.size() * 4));
            HIP_TRY(h, hipMemcpy(h->d_dxslab, slab.data(), slab.size() * 4, hipMemcpyHostToDevice));
        }
        h->ready = true;
        return WRNN_OK;
    }
    // pack and upload
    if (h->max_rows >= 1) {
        std::vector<float> slab((size_t)h->G * h->s.total);
        for (int w = 0; w < h->G; ++w) pack_slab(*h, w, slab.data() + (size_t)w * h->s.total);
        if (!h->d_slab) HIP_TRY(h, hipMalloc(&h->d_slab, slab.size() * 4));
        HIP_TRY(h, hipMemcpy(h->d_slab, slab.data(), slab.size() * 4, hipMemcpyHostToDevice));
    }
    const auto &IW = h->w.at("I.weight");
    const auto &Ib = h->w.at("I.bias");
    if (!h->d_IW) HIP_TRY(h, hipMalloc(&h->d_IW, IW.size() * 4));
    if (!h->d_Ib) HIP_TRY(h, hipMalloc(&h->d_Ib, Ib.size() * 4));
    HIP_TRY(h, hipMemcpy(h->d_IW, IW.data(), IW.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(h, hipMemcpy(h->d_Ib, Ib.data(), Ib.size() * 4, hipMemcpyHostToDevice));
    // rows kernel: block-sparse GRU weights (pruning.py) are kept as nonzero 4x4 blocks when the
    // block density is <= 1/2 (WRNN_SPARSE=0 keeps them dense)
    {
        const int R = h->cfg.rnn_dims;
        int nbmax = 0;
        double density = 1.0;
        const char *sp_env = std::getenv("WRNN_SPARSE");
        if (R % 4 == 0 && R / 4 <= h->num_cus && !(sp_env && std::string(sp_env) == "0"))
            block_stats(*h, &nbmax, &density);
        set_rows_partition(*h, density <= 0.5 ? std::max(nbmax, 1) : 0);
        if (h->rows_ok) {
            int per_cu = 0;
            HIP_TRY(h, rows_occupancy(&per_cu, rows_lds_bytes(*h, 1, 1)));
            if (per_cu * h->num_cus < h->rG) h->rows_ok = false;
        }
        if (h->max_rows < 1 && !h->rows_ok)
            return fail(h, WRNN_EUNSUPPORTED, "these dims fit neither kernel's LDS layout with dense GRU weights "
                                              "(block-sparse 4x4 GRU weights would, see pruning.py)");
    }
    if (h->rows_ok) {
        std::vector<float> rslab((size_t)h->rG * h->rs.total);
        for (int w = 0; w < h->rG; ++w) pack_rows_slab(*h, w, rslab.data() + (size_t)w * h->rs.total);
        if (h->d_rslab) HIP_TRY(h, hipFree(h->d_rslab));
        HIP_TRY(h, hipMalloc(&h->d_rslab, rslab.size() * 4));
        HIP_TRY(h, hipMemcpy(h->d_rslab, rslab.data(), rslab.size() * 4, hipMemcpyHostToDevice));
        std::vector<float> Wt((size_t)h->rG * h->NT * rows_terms_kx(*h));
        if (rows_terms_composed(*h)) pack_terms_weights_composed(*h, Wt.data());
        else pack_terms_weights(*h, Wt.data());
        if (h->d_Wt) HIP_TRY(h, hipFree(h->d_Wt));
        HIP_TRY(h, hipMalloc(&h->d_Wt, Wt.size() * 4));
        HIP_TRY(h, hipMemcpy(h->d_Wt, Wt.data(), Wt.size() * 4, hipMemcpyHostToDevice));
    }
    if (h->g2.ok && !h->sparse) {
        PartScope ps(*h, h->g2, true);
        std::vector<float> rslab((size_t)h->rG * h->rs.total);
        for (int w = 0; w < h->rG; ++w) pack_rows_slab(*h, w, rslab.data() + (size_t)w * h->rs.total);
        if (h->d_rslab) HIP_TRY(h, hipFree(h->d_rslab));
        h->d_rslab = nullptr;
        HIP_TRY(h, hipMalloc(&h->d_rslab, rslab.size() * 4));
        HIP_TRY(h, hipMemcpy(h->d_rslab, rslab.data(), rslab.size() * 4, hipMemcpyHostToDevice));
        std::vector<float> Wt((size_t)h->rG * h->NT * rows_terms_kx(*h));
        if (rows_terms_composed(*h)) pack_terms_weights_composed(*h, Wt.data());
        else pack_terms_weights(*h, Wt.data());
        if (h->d_Wt) HIP_TRY(h, hipFree(h->d_Wt));
        h->d_Wt = nullptr;
        HIP_TRY(h, hipMalloc(&h->d_Wt, Wt.size() * 4));
        HIP_TRY(h, hipMemcpy(h->d_Wt, Wt.data(), Wt.size() * 4, hipMemcpyHostToDevice));
    }
    if (h->split_ok) {
        std::vector<float> gs, fs, Wt;
        pack_split_slabs(*h, gs, fs);
        pack_split_terms_weights(*h, Wt);
        for (auto pr : {std::make_pair(&h->d_sgslab, &gs), std::make_pair(&h->d_sfslab, &fs),
                        std::make_pair(&h->d_sWt, &Wt)}) {
            if (*pr.first) HIP_TRY(h, hipFree(*pr.first));
            *pr.first = nullptr;
            HIP_TRY(h, hipMalloc(pr.first, pr.second->size() * 4));
            HIP_TRY(h, hipMemcpy(*pr.first, pr.second->data(), pr.second->size() * 4, hipMemcpyHostToDevice));
        }
    }
    if (h->xcd_ok || h->xcdm_ok) {   // (the many-row kernel shares the terms GEMM; RAW has no xcd slab)
        std::vector<float> slab, Wt;
        if (h->xcd_ok) pack_xcd_slab(*h, slab);
        else slab.assign(4, 0.0f);
        pack_xcd_terms_weights(*h, Wt);
        for (auto pr : {std::make_pair(&h->d_xslab, &slab), std::make_pair(&h->d_xWt, &Wt)}) {
            if (*pr.first) HIP_TRY(h, hipFree(*pr.first));
            *pr.first = nullptr;
            HIP_TRY(h, hipMalloc(pr.first, pr.second->size() * 4));
            HIP_TRY(h, hipMemcpy(*pr.first, pr.second->data(), pr.second->size() * 4, hipMemcpyHostToDevice));
        }
    }
    if (h->xcdm_ok) {
        std::vector<float> slab, Wm;
        pack_xcdm_terms_weights(*h, Wm);
        if (h->d_xmWt) HIP_TRY(h, hipFree(h->d_xmWt));
        h->d_xmWt = nullptr;
        HIP_TRY(h, hipMalloc(&h->d_xmWt, Wm.size() * 4));
        HIP_TRY(h, hipMemcpy(h->d_xmWt, Wm.data(), Wm.size() * 4, hipMemcpyHostToDevice));
        pack_xcdm_slab(*h, slab);
        if (h->d_xmslab) HIP_TRY(h, hipFree(h->d_xmslab));
        h->d_xmslab = nullptr;
        HIP_TRY(h, hipMalloc(&h->d_xmslab, slab.size() * 4));
        HIP_TRY(h, hipMemcpy(h->d_xmslab, slab.data(), slab.size() * 4, hipMemcpyHostToDevice));
    }
    h->xcds_ok = false;
    if (h->xcds_cap) {
        const char *sp_env = std::getenv("WRNN_SPARSE");
        const int nbmax = (sp_env && std::string(sp_env) == "0") ? kSNB + 1 : xcds_nbmax(*h);
        if (h->sparse && nbmax <= kSNB) {
            std::vector<float> slab, Wt;
            pack_xcds_slab(*h, slab);
            pack_xcds_terms_weights(*h, Wt);
            for (auto pr : {std::make_pair(&h->d_xslab, &slab), std::make_pair(&h->d_xWt, &Wt)}) {
                if (*pr.first) HIP_TRY(h, hipFree(*pr.first));
                *pr.first = nullptr;
                HIP_TRY(h, hipMalloc(pr.first, pr.second->size() * 4));
                HIP_TRY(h, hipMemcpy(*pr.first, pr.second->data(), pr.second->size() * 4, hipMemcpyHostToDevice));
            }
            h->xcds_ok = true;
        }
    }
    h->ready = true;
    return WRNN_OK;
}

constexpr int kXcdDefaultRows = 48;
constexpr int kXcdmMinRows = 9;

// The loop path for B rows (WRNN_PATH=xcd|xcdm|split|latency|rows forces one: tests, benchmarks).
enum LoopPath { P_LATENCY = 1, P_ROWS = 2, P_DM = 3, P_SPLIT = 4, P_XCD = 5, P_XCDS = 6, P_XCDM = 7, P_DX = 8 };
static LoopPath choose_path(const wrnn_t *h, int B) {
    const char *path_env = std::getenv("WRNN_PATH");
    const std::string pe = path_env ? path_env : "";
    // deepmind hidden 896 / quantisation 256: the XCD-resident kernel (WRNN_PATH=rows: the multi-row one)
    if (h->dm) return h->dx_ok && pe != "rows" ? P_DX : P_DM;
    bool rows = h->max_rows < 1 || B > h->max_rows;
    if (pe == "rows") rows = true;
    if (pe == "latency" && h->max_rows >= 1) rows = false;
    if (rows && !h->rows_ok) rows = false;
    // MoL rnn / fc 512 up to kXcdDefaultRows rows: the XCD-resident kernel (8 rows per launch;
    // beyond that the multi-row kernel's throughput wins)
    // MoL rnn / fc 512, more than kXcdmMinRows rows: the many-row XCD-resident kernel (MFMA)
    // (RAW 512-class: the many-row kernel for every row count — it is the only XCD-resident RAW one)
    if (h->xcdm_ok && (pe == "xcdm" || (pe.empty() && (B >= kXcdmMinRows || h->cfg.mode == WRNN_MODE_RAW))))
        return P_XCDM;
    if (h->xcd_ok && (pe == "xcd" || (pe.empty() && B <= kXcdDefaultRows))) return P_XCD;
    // MoL rnn 896 with block-sparse GRU weights likewise: the XCD-resident sparse kernel
    if (h->xcds_ok && (pe == "xcd" || (pe.empty() && B <= kXcdDefaultRows))) return P_XCDS;
    if (h->split_ok && (pe == "split" || (pe.empty() && B == 1))) return P_SPLIT;
    return rows ? P_ROWS : P_LATENCY;
}

// One loop run over the chosen path, between the two timing events.  `fs` (frame-rate terms)
// only for the XCD-resident paths.
static int run_loop(wrnn_t *h, LoopPath path, const float *cond, const FrameSrc *fs, int B, int L, const float *noise,
             uint64_t seed, int64_t row_offset, float *out, int32_t *labels, hipStream_t st) {
    HIP_TRY(h, hipMemsetAsync(h->d_ctl, 0, kCtlWords * sizeof(int), st));
    HIP_TRY(h, hipEventRecord(h->ev0, st));
    h->last_path = path == P_ROWS && h->rows_gw ? 9 : path == P_DM && h->dm_gw ? 10 : (int)path;
    int rc = WRNN_OK;
    switch (path) {
        case P_DX: rc = generate_dx(h, B, L, noise, seed, row_offset, out, labels, st); break;
        case P_DM: rc = generate_dm(h, B, L, noise, seed, row_offset, out, labels, st); break;
        case P_XCDM: rc = generate_xcdm(h, cond, fs, B, L, noise, seed, row_offset, out, labels, st); break;
        case P_XCD: rc = generate_xcd(h, cond, fs, B, L, noise, seed, row_offset, out, st); break;
        case P_XCDS: rc = generate_xcds(h, cond, fs, B, L, noise, seed, row_offset, out, st); break;
        case P_SPLIT: rc = generate_split(h, cond, B, L, noise, seed, row_offset, out, st); break;
        case P_ROWS: rc = generate_rows(h, cond, B, L, noise, seed, row_offset, out, labels, st); break;
        default: rc = generate_latency(h, cond, B, L, noise, seed, row_offset, out, labels, st); break;
    }
    if (rc != WRNN_OK) return rc;
    HIP_TRY(h, hipEventRecord(h->ev1, st));
    h->timed = true;
    return WRNN_OK;
}

int wrnn_generate(wrnn_t *h, const float *cond, int B, int L, const float *noise, uint64_t seed,
                  int64_t row_offset, float *out, int32_t *labels, void *stream) {
    if (!h) return WRNN_EINVAL;
    if (!h->ready) return fail(h, WRNN_ENOWEIGHTS, "weights not (fully) set");
    if (B <= 0 || L <= 0 || !out || (!cond && !h->dm)) return fail(h, WRNN_EINVAL, "need B > 0, L > 0, cond and out");
    if (labels && h->cfg.mode == WRNN_MODE_MOL) return fail(h, WRNN_EINVAL, "labels are a RAW / DM output");
    HIP_TRY(h, hipSetDevice(h->device));
    return run_loop(h, choose_path(h, B), cond, nullptr, B, L, noise, seed, row_offset, out, labels,
                    (hipStream_t)stream);
}

int wrnn_frame_weights(const wrnn_upsample_cfg *ucfg, int *hop, int *nJ, int *jlo, float *coef, int coef_cap) {
    if (!ucfg || ucfg->n_scales < 1 || ucfg->n_scales > 4) return WRNN_EINVAL;
    for (int i = 0; i < ucfg->n_scales; ++i)
        if (ucfg->scales[i] < 1 || !ucfg->taps[i]) return WRNN_EINVAL;
    int hh = 1, nj = 1, jl = 0;
    std::vector<float> c;
    if (!frame_weights(*ucfg, &hh, &nj, &jl, c)) return WRNN_EUNSUPPORTED;
    if (hop) *hop = hh;
    if (nJ) *nJ = nj;
    if (jlo) *jlo = jl;
    if (coef) {
        if (coef_cap < (int)c.size()) return WRNN_EINVAL;
        std::memcpy(coef, c.data(), c.size() * sizeof(float));
    }
    return WRNN_OK;
}

int wrnn_generate_frames(wrnn_t *h, const wrnn_upsample_cfg *ucfg, const float *mel, const float *aux, int U, int T,
                         int target, int overlap, const float *noise, uint64_t seed, int64_t row_offset, float *out,
                         int32_t *labels, void *stream) {
    return wrnn_generate_frames_rows(h, ucfg, mel, aux, U, T, target, overlap, 0, -1, noise, seed, row_offset, out,
                                     labels, stream);
}

// row_count < 0: every row of the launch (wrnn_generate_frames)
int wrnn_generate_frames_rows(wrnn_t *h, const wrnn_upsample_cfg *ucfg, const float *mel, const float *aux, int U,
                              int T, int target, int overlap, int row_begin, int row_count, const float *noise,
                              uint64_t seed, int64_t row_offset, float *out, int32_t *labels, void *stream) {
    if (!h) return WRNN_EINVAL;
    if (!h->ready) return fail(h, WRNN_ENOWEIGHTS, "weights not (fully) set");
    if (h->dm) return fail(h, WRNN_EINVAL, "deepmind handles take no conditioning (wrnn_generate)");
    if (!ucfg || !mel || !out || U <= 0 || T <= 0) return fail(h, WRNN_EINVAL, "need ucfg, mel, out, U > 0, T > 0");
    if (labels && h->cfg.mode == WRNN_MODE_MOL) return fail(h, WRNN_EINVAL, "labels are a RAW / DM output");
    if (ucfg->feat_dims != h->cfg.feat_dims || ucfg->res_out_dims != h->CD - h->cfg.feat_dims)
        return fail(h, WRNN_EINVAL, "upsample config does not match the handle's feat / aux dims");
    if (ucfg->res_out_dims > 0 && !aux) return fail(h, WRNN_EINVAL, "need aux (MelResNet output)");
    int L = 0, Ball = 0;
    if (int rc = wrnn_cond_shape(ucfg, U, T, target, overlap, &L, &Ball))
        return fail(h, rc, std::string("conditioning shape: ") + wrnn_cond_last_error());
    if (row_count < 0) {
        row_begin = 0;
        row_count = Ball;
    }
    if (row_begin < 0 || row_count < 1 || row_begin + row_count > Ball)
        return fail(h, WRNN_EINVAL, "rows [row_begin, row_begin + row_count) outside the launch's " + std::to_string(Ball));
    const int B = row_count;
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    const LoopPath path = choose_path(h, B);
    FrameSrc fs;
    std::vector<float> coef;
    bool frames = (path == P_XCD || path == P_XCDS || path == P_XCDM) && std::getenv("WRNN_NO_FRAME_TERMS") == nullptr &&
                  frame_weights(*ucfg, &fs.hop, &fs.nJ, &fs.jlo, coef);
    if (frames) {
        const int N = kXcdWgs * (path == P_XCD ? kXTerms : path == P_XCDS ? kSTerms : kMRing);
        frames = N % 4 == 0;
    }
    if (!frames) {   // the per-sample conditioning (wrnn_upsample_pack) into a handle workspace
        const size_t rec = (size_t)h->CD * sizeof(float);
        if (grow(h, h->d_cond, h->cond_cap, (size_t)L * (Ball + (B < Ball ? B : 0)) * h->CD)) return WRNN_EHIP;
        if (int rc = wrnn_upsample_pack(ucfg, mel, aux, U, T, target, overlap, h->d_cond, stream))
            return fail(h, rc, std::string("upsample_pack: ") + wrnn_cond_last_error());
        const float *cond = h->d_cond;
        if (B < Ball) {   // the rows' records, compacted after the launch's [L][Ball] block
            float *sub = h->d_cond + (size_t)L * Ball * h->CD;
            HIP_TRY(h, hipMemcpy2DAsync(sub, B * rec, h->d_cond + (size_t)row_begin * h->CD, Ball * rec, B * rec, L,
                                        hipMemcpyDeviceToDevice, st));
            cond = sub;
        }
        return run_loop(h, path, cond, nullptr, B, L, noise, seed, row_offset, out, labels, st);
    }
    if (coef != h->coef_host) {
        if (grow(h, h->d_coef, h->coef_cap, coef.size())) return WRNN_EHIP;
        HIP_TRY(h, hipMemcpyAsync(h->d_coef, coef.data(), coef.size() * 4, hipMemcpyHostToDevice, st));
        HIP_TRY(h, hipStreamSynchronize(st));   // `coef` is a local: the copy completes before it goes
        h->coef_host = coef;
    }
    fs.mel = mel;
    fs.aux = aux;
    fs.U = U;
    fs.NF = T;
    fs.nf = Ball / U;
    fs.rb = row_begin;
    fs.stride = target > 0 ? target + overlap : 0;
    fs.coef = h->d_coef;
    return run_loop(h, path, nullptr, &fs, B, L, noise, seed, row_offset, out, labels, st);
}

int wrnn_check(wrnn_t *h, void *stream) {
    if (!h) return WRNN_EINVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipStreamSynchronize((hipStream_t)stream));
    int ctl[kCtlWords];
    HIP_TRY(h, hipMemcpy(ctl, h->d_ctl, sizeof(ctl), hipMemcpyDeviceToHost));
    if (ctl[1] != 0) {
        static const char *lat_hops[] = {"q1", "h2", "f1", "f2", "logits", "gru1-terms", "gru1-terms"};
        static const char *row_hops[] = {"h1", "h2", "f1", "f2", "logits", "x"};
        const int hop = ctl[3];
        static const char *dm_hops[] = {"h_coarse", "o1", "coarse logits", "h_fine", "o3", "fine logits",
                                        "coarse label", "fine label"};
        static const char *split_hops[] = {"y", "f1", "f2", "h2", "h2", "gru1-terms", "gru1-terms"};
        static const char *xcd_hops[] = {"y", "f1", "f2", "h2", "gru1-terms", "gru1-terms"};
        static const char *xcdm_hops[] = {"h1", "y", "h2", "f1", "f2 (partial logits)", "x", "logits"};
        const int lp = h->last_path;
        const char *name = lp == 8 || lp == 3 || lp == 10 ? (hop >= 0 && hop < 8 ? dm_hops[hop] : "?")
                           : lp == 2 || lp == 9         ? (hop >= 0 && hop < 6 ? row_hops[hop] : "?")
                           : lp == 7                    ? (hop >= 0 && hop < 7 ? xcdm_hops[hop] : "?")
                           : lp >= 5                    ? (hop >= 0 && hop < 6 ? xcd_hops[hop] : "?")
                           : lp == 4                    ? (hop >= 0 && hop < 7 ? split_hops[hop] : "?")
                                                        : (hop >= 0 && hop < 7 ? lat_hops[hop] : "?");
        return fail(h, WRNN_ETIMEOUT,
                    "persistent kernel aborted: wait on hand-off '" + std::string(name) +
                        "' at step " + std::to_string(ctl[2]) + " in workgroup " + std::to_string(ctl[4]) +
                        " exceeded the timeout (grid not co-resident, or a fault)");
    }
    return WRNN_OK;
}

int wrnn_elapsed_ms(wrnn_t *h, float *ms) {
    if (!h || !ms) return WRNN_EINVAL;
    if (!h->timed) return fail(h, WRNN_EINVAL, "no wrnn_generate recorded yet");
    HIP_TRY(h, hipEventSynchronize(h->ev1));
    HIP_TRY(h, hipEventElapsedTime(ms, h->ev0, h->ev1));
    return WRNN_OK;
}

int wrnn_query(const wrnn_t *h, wrnn_info *info) {
    if (!h || !info) return WRNN_EINVAL;
    if (h->dm) {
        *info = wrnn_info{};
        info->grid = h->G;
        info->units_rnn = h->dmU;
        info->units_fc = h->dmUO;
        info->units_cls = h->dmUO2;
        info->lds_bytes = (int)dm_lds_bytes(*h, 1, 1);
        info->slab_floats = h->ds.total;
        info->num_cus = h->num_cus;
        info->rows_grid = h->G;
        info->rows_units_rnn = h->dmU;
        info->last_path = h->last_path;
        info->xcd_rows = h->dx_ok ? kDxRowsMax : 0;
        return WRNN_OK;
    }
    const bool rows_only = h->max_rows < 1;      // e.g. rnn 896 with block-sparse GRU weights
    info->grid = rows_only ? h->rG : h->G;
    info->units_rnn = rows_only ? h->rU : h->U;
    info->units_fc = rows_only ? h->rUF : h->UF;
    info->units_cls = rows_only ? h->rUC : h->UC;
    info->max_rows = h->max_rows;
    info->lds_bytes = (int)(rows_only ? rows_lds_bytes(*h, 1, 1) : lds_bytes_for(*h, h->max_rows));
    info->slab_floats = rows_only ? h->rs.total : h->s.total;
    info->rows_grid = h->rows_ok ? h->rG : 0;
    info->rows_units_rnn = h->rows_ok ? h->rU : 0;
    info->sparse_blocks = h->rows_ok ? h->rs.nbmax : 0;
    info->num_cus = h->num_cus;
    info->split_grid = h->split_ok ? h->sGg + h->sGf : 0;
    info->last_path = h->last_path;
    info->xcd_rows = (h->xcd_ok || h->xcds_ok) ? kXcds : 0;
    info->xcdm_rows = h->xcdm_ok ? kXcds * 4 * h->xcdm_nq : 0;
    return WRNN_OK;
}

const char *wrnn_last_error(const wrnn_t *h) { return h ? h->err.c_str() : "null handle"; }

int wrnn_philox_draws(uint64_t seed, int64_t row_offset, int rows, int step0, int steps, int K, int mode, float *out,
                      void *stream) {
    if (!out || rows < 1 || steps < 1 || K < 1 || step0 < 0)
        return cond_fail(WRNN_EINVAL, "need out, rows >= 1, steps >= 1, K >= 1, step0 >= 0");
    if (mode != WRNN_MODE_RAW && mode != WRNN_MODE_MOL && mode != WRNN_MODE_DM)
        return cond_fail(WRNN_EINVAL, "unknown mode");
    if ((long long)steps * rows * K > (1LL << 31) - 256) return cond_fail(WRNN_EINVAL, "too many draws for one call");
    if ((long long)step0 + steps > (1LL << 32)) return cond_fail(WRNN_EINVAL, "step index past 2^32");
    if (launch_philox_fill(out, seed, row_offset, rows, step0, steps, K, mode == WRNN_MODE_MOL ? 1 : 0,
                           (hipStream_t)stream) != hipSuccess)
        return cond_fail(WRNN_EHIP, "philox fill launch failed");
    return WRNN_OK;
}

void wrnn_destroy(wrnn_t *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    for (void *p : {(void *)h->d_slab, (void *)h->d_IW, (void *)h->d_Ib, (void *)h->d_cI, (void *)h->d_xg,
                    (void *)h->d_ctl, (void *)h->d_rslab, (void *)h->d_Wt, (void *)h->d_X, (void *)h->d_T,
                    (void *)h->d_act, (void *)h->d_state, (void *)h->d_flags, (void *)h->d_xr, (void *)h->d_dmslab,
                    (void *)h->d_dmflags, (void *)h->d_dmxg, (void *)h->d_sgslab, (void *)h->d_sfslab,
                    (void *)h->d_sWt, (void *)h->g2.d_slab, (void *)h->g2.d_Wt, (void *)h->dm2.d_slab,
                    (void *)h->d_gact, (void *)h->d_xslab, (void *)h->d_xWt, (void *)h->d_xstate, (void *)h->d_xgx,
                    (void *)h->d_members, (void *)h->d_xmslab, (void *)h->d_xmstate, (void *)h->d_xmxg, (void *)h->d_xmnoise,
                    (void *)h->d_xmWt, (void *)h->d_coef, (void *)h->d_FT, (void *)h->d_AT, (void *)h->d_frec,
                    (void *)h->d_cond,
                    (void *)h->d_dxslab, (void *)h->d_dxstate, (void *)h->d_dxnoise, (void *)h->d_dxxg})
        if (p) (void)hipFree(p);
    if (h->blas) (void)rocblas_destroy_handle(h->blas);
    delete h;
}

}  // extern "C"
