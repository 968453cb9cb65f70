// frame_terms.hip — the persistent kernels' conditioning terms formed at FRAME rate.
//
// Every MoL / RAW persistent kernel reads, per loop row and step, terms = W·[mel_up(p) | aux(p) | 1]
// (the I layer of fatchord_version.py:201-206 folded with the input halves of both GRUs, fc1 and
// fc2 into one matrix W, capi.cpp).  The reference's UpsampleNetwork (:64-89) is linear and, in
// units of frames, shift-invariant: with f = p div hop and φ = p mod hop,
//   mel_up(p) = Σ_k coef[φ][k] · mel[f + k + jlo],   coef[φ][k] = κ(φ − hop·(k + jlo)),
// κ the Stretch2d/Conv2d cascade's response to one frame (the cascade's zero padding is the
// frame-level zero padding once pad_tensor's pad frames cover κ's reach), and aux(p) = aux[f]
// (resnet_stretch, :83).  Hence
//   terms(p) = Σ_k coef[φ][k] · FT[f + k] + AT[f],
//   FT[i] = W·[mel[i + jlo] | 0 | 0],   AT[f] = W·[0 | aux[f] | 1],   AT[n_frames] = W·[0 | 0 | 1]
// (the last row: steps past the utterance, fold_with_overlap's zero tail, :317-330).  The terms
// GEMM runs over the n_frames frames instead of the hop·n_frames samples (hop 275: 275× fewer
// flops); what is left per sample is this nJ-tap sum over cached rows, an HBM-write-bound pass.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wrnn {

// Frame-level conditioning records [frames][U][CD] for the path's own GEMM-input packer
// (pack_cond_input_kernel): kind 0 → record i = [mel[:, i + jlo] (0 outside [0, NF)) | 0 …],
// kind 1 → record f = [0 … | aux[:, f]] (f == NF: all zero).  mel [U][feat][NF], aux [U][A4][NF].
__global__ void frame_cond_kernel(const float *__restrict__ mel, const float *__restrict__ aux, int U, int feat, int A4,
                                  int NF, int frames, int jlo, int kind, float *__restrict__ rec) {
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);   // record (frame · U + u), one wave each
    if (m >= frames * U) return;
    const int i = m / U, u = m - i * U;
    const int CD = feat + A4;
    float *dst = rec + (size_t)m * CD;
    for (int c = threadIdx.x & 63; c < CD; c += 64) {
        float v = 0.0f;
        if (kind == 0) {
            const int fr = i + jlo;
            if (c < feat && fr >= 0 && fr < NF) v = mel[((size_t)u * feat + c) * NF + fr];
        } else if (c >= feat && i < NF) {
            v = aux[((size_t)u * A4 + (c - feat)) * NF + i];
        }
        dst[c] = v;
    }
}

hipError_t launch_frame_cond(const float *mel, const float *aux, int U, int feat, int A4, int NF, int frames, int jlo,
                             int kind, float *rec, hipStream_t st) {
    const int M = frames * U;
    hipLaunchKernelGGL(frame_cond_kernel, dim3((M + 3) / 4), dim3(256), 0, st, mel, aux, U, feat, A4, NF, frames, jlo,
                       kind, rec);
    return hipGetLastError();
}

struct InterpArgs {
    const float *FT;      // [NFF][U][N]   W·(one mel frame)
    const float *AT;      // [NF + 1][U][N] W·(aux frame, ones); row NF: W·(ones)
    const float *coef;    // [hop][nJ]
    float *T;             // [nt · nb][N]  record (t − t0)·nb + k
    int N, U, NF, NFF, hop, nJ;
    int nf, stride;       // loop row r: utterance r / nf, first step (r % nf)·stride
    int b0, nb, t0, nt;
};

constexpr int kInterpThreads = 256;
constexpr int kInterpSteps = 32;   // consecutive steps of one row per workgroup: a frame's rows (hop ≥ 32
                                   // steps) are loaded once and stay in registers
constexpr int kInterpMaxJ = 8;

// One workgroup: a 1 024-float column slice (a float4 per lane) of kInterpSteps consecutive steps of
// ONE loop row.  The frame rows FT[f .. f + nJ) and AT[f] are reloaded only when the step crosses
// into another frame (wave-uniform branch), so the pass reads ≈ 6/32 of what it writes: it is
// bound by the terms it writes, not by re-reading cached rows (8 records of 8 rows per workgroup
// reloaded all six rows per record: 2.2 TB/s effective).
__global__ __launch_bounds__(kInterpThreads) void terms_interp_kernel(InterpArgs a) {
    const int c4 = blockIdx.y * kInterpThreads + threadIdx.x;   // float4 column
    if (4 * c4 >= a.N) return;
    const int nblk = (a.nt + kInterpSteps - 1) / kInterpSteps;
    const int k = blockIdx.x / nblk, tb = (blockIdx.x - k * nblk) * kInterpSteps;
    const int r = a.b0 + k, u = r / a.nf;
    const int s0 = (r - u * a.nf) * a.stride + a.t0;            // utterance position of step t0
    const int L_utt = a.NF * a.hop;
    const size_t rs = (size_t)a.U * a.N;                         // frame-row stride
    const float *A0 = a.AT + (size_t)u * a.N + 4 * c4, *F0 = a.FT + (size_t)u * a.N + 4 * c4;
    float4 fr[kInterpMaxJ], ar = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int loaded = -1;
    for (int i = 0; i < kInterpSteps; ++i) {
        const int tl = tb + i;
        if (tl >= a.nt) break;
        const int p = s0 + tl;
        const int f = p < L_utt ? p / a.hop : a.NF;               // a.NF: past the utterance (W·[0 | 0 | 1])
        if (f != loaded) {
            ar = *reinterpret_cast<const float4 *>(A0 + (size_t)f * rs);
            if (f < a.NF) {
#pragma unroll
                for (int j = 0; j < kInterpMaxJ; ++j)
                    if (j < a.nJ) fr[j] = *reinterpret_cast<const float4 *>(F0 + (size_t)(f + j) * rs);
            }
            loaded = f;
        }
        float4 acc = ar;
        if (f < a.NF) {
            const float *cf = a.coef + (size_t)(p - f * a.hop) * a.nJ;
#pragma unroll
            for (int j = 0; j < kInterpMaxJ; ++j) {
                if (j < a.nJ) {
                    const float w = cf[j];
                    acc.x = fmaf(w, fr[j].x, acc.x);
                    acc.y = fmaf(w, fr[j].y, acc.y);
                    acc.z = fmaf(w, fr[j].z, acc.z);
                    acc.w = fmaf(w, fr[j].w, acc.w);
                }
            }
        }
        *reinterpret_cast<float4 *>(a.T + ((size_t)tl * a.nb + k) * a.N + 4 * c4) = acc;
    }
}

// N % 4 == 0 and nJ <= kInterpMaxJ (the host checks both before choosing the frame path)
hipError_t launch_terms_interp(const float *FT, const float *AT, const float *coef, float *T, int N, int U, int NF,
                               int NFF, int hop, int nJ, int nf, int stride, int b0, int nb, int t0, int nt,
                               hipStream_t st) {
    InterpArgs a{FT, AT, coef, T, N, U, NF, NFF, hop, nJ, nf, stride, b0, nb, t0, nt};
    const dim3 grid(nb * ((nt + kInterpSteps - 1) / kInterpSteps), (N / 4 + kInterpThreads - 1) / kInterpThreads);
    hipLaunchKernelGGL(terms_interp_kernel, grid, dim3(kInterpThreads), 0, st, a);
    return hipGetLastError();
}

}  // namespace wrnn
