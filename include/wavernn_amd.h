/*
 * wavernn_amd.h — C-ABI of the MI355X-native WaveRNN generation path.
 *
 * The reference has no FFI: its hot path is the Python method
 *   WaveRNN.generate(mels, save_path, batched, target, overlap, mu_law)
 *   (/root/reference/models/fatchord_version.py:169-264)
 * whose per-sample loop (:201-241) dispatches ~40 eager torch ops per step.  This ABI is
 * what that method binds instead (wavernn_amd/fatchord_version.py does it via ctypes; see
 * INTEGRATION.md for the binding a reference maintainer would add).  Each entry point names
 * the reference code it replaces.
 *
 * Conventions: plain pointers and sizes only; return 0 or a negative WRNN_E* code; no
 * exception crosses the ABI; device pointers are HIP device pointers on the handle's device;
 * `stream` is a hipStream_t (NULL = default stream); calls are asynchronous on that stream
 * except where stated; one handle per device, not thread-safe.
 */
#ifndef WAVERNN_AMD_H
#define WAVERNN_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WRNN_ABI_VERSION 6

enum wrnn_status {
    WRNN_OK = 0,
    WRNN_EINVAL = -1,        /* bad argument / shape (message in wrnn_last_error)            */
    WRNN_EHIP = -2,          /* a HIP runtime call failed                                    */
    WRNN_ENOWEIGHTS = -3,    /* wrnn_generate before every required tensor was set           */
    WRNN_ETIMEOUT = -4,      /* a persistent-kernel wait exceeded its bound (kernel aborted)  */
    WRNN_ENOMEM = -5,
    WRNN_EUNSUPPORTED = -6,  /* dims / device the kernel cannot run (e.g. LDS or residency)  */
};

enum wrnn_mode {             /* fatchord_version.py:97-104 */
    WRNN_MODE_RAW = 0,       /* softmax over 2**bits classes, Categorical sample (:231-237) */
    WRNN_MODE_MOL = 1,       /* 30-way mixture of logistics (:225-229)                       */
    WRNN_MODE_DM = 2,        /* deepmind_version.py: dual coarse/fine 8-bit softmax (:75-165);
                                rnn_dims = hidden_size, n_classes = quantisation; the fc/aux/
                                feat dims are unused (no conditioning)                         */
};

typedef struct wrnn_ctx wrnn_t;

/* Model dims — the WaveRNN constructor arguments that shape the loop
 * (fatchord_version.py:93-123; aux_dims = res_out_dims / 4 at :110). */
typedef struct {
    int32_t abi_version;     /* must be WRNN_ABI_VERSION */
    int32_t mode;            /* enum wrnn_mode */
    int32_t rnn_dims;
    int32_t fc_dims;
    int32_t aux_dims;
    int32_t feat_dims;       /* num_mels */
    int32_t n_classes;       /* 2**bits (RAW) or 30 (MOL) */
    int32_t grid;            /* workgroups of the persistent kernel; 0 = auto (one per CU) */
    int32_t timeout_ms;      /* bound on any single in-kernel wait; 0 = default (2000 ms) */
} wrnn_config;

/* One named weight, named exactly as the reference state_dict key
 * (e.g. "rnn1.weight_ih_l0"), fp32 row-major in the reference shape. */
typedef struct {
    const char *name;
    const float *data;
    int64_t numel;
    int32_t on_device;       /* 1: `data` is a device pointer, 0: host pointer */
} wrnn_tensor;

/* Launch geometry chosen for the handle (read-only).  Kernels: the XCD-resident kernel (MoL
 * rnn/fc 512, up to 8 rows per launch, one row on each XCD's 32 CUs), its many-row form (up to
 * 16 rows per XCD on the matrix cores, 128 per launch), the role-split kernel
 * (one MoL row), the per-row latency kernel (rows in LDS, used while B <= max_rows) and the
 * multi-row kernel (rows through HBM). */
typedef struct {
    int32_t grid;            /* workgroups (all co-resident, one persistent launch) */
    int32_t units_rnn;       /* hidden units per workgroup (GRU rows ×3)            */
    int32_t units_fc;        /* fc1/fc2 rows per workgroup                          */
    int32_t units_cls;       /* fc3 rows per workgroup (RAW; MOL computes all 30)   */
    int32_t max_rows;        /* rows one latency-kernel launch holds (0: multi-row kernel only) */
    int32_t lds_bytes;       /* dynamic LDS per workgroup at max_rows                */
    int32_t slab_floats;     /* resident weight floats per workgroup                 */
    int32_t num_cus;
    int32_t rows_grid;       /* multi-row kernel: workgroups (0: unavailable)        */
    int32_t rows_units_rnn;  /*                   hidden units per workgroup         */
    int32_t sparse_blocks;   /*                   max nonzero 4x4 blocks per gate block-row when
                                                  the GRU weights are block-sparse, else 0 */
    int32_t split_grid;      /* batch-1 MoL role-split kernel: GRU + FC workgroups (0: unavailable) */
    int32_t last_path;       /* kernel of the last wrnn_generate: 1 latency, 2 multi-row,
                                3 deepmind, 4 role-split, 5 XCD-resident, 6 XCD-resident
                                block-sparse rnn 896, 7 XCD-resident many-row, 8 XCD-resident
                                deepmind, 9 multi-row with the weights streamed from HBM (dense
                                weights beyond LDS), 10 deepmind streamed (0: none yet) */
    int32_t xcd_rows;        /* XCD-resident kernel, rows per launch (0: unavailable).  RAW/MOL
                                handles: the one-row-per-XCD kernel (dense rnn 512, or rnn 896
                                with block-sparse GRU weights once they are set), 8.  DM handles
                                (ABI 5): the XCD-resident deepmind kernel (hidden 896 / Q 256,
                                4 rows per XCD), 32. */
    int32_t xcdm_rows;       /* XCD-resident many-row kernel (MoL rnn/fc 512): rows per launch
                                (0: unavailable)                                           (ABI 5) */
} wrnn_info;

/* Create a handle on `device` (replaces WaveRNN.__init__ for the loop's dims,
 * fatchord_version.py:93-129).  Synchronous.  On failure *out may still hold a handle so
 * the caller can read wrnn_last_error(); release it with wrnn_destroy. */
int wrnn_create(const wrnn_config *cfg, int device, wrnn_t **out);

/* Load weights by reference state_dict name (replaces WaveRNN.load → load_state_dict,
 * fatchord_version.py:414-417, for the loop's tensors: I.*, rnn1.*, rnn2.*, fc1-3.*).
 * Copies and packs into the kernel's per-workgroup layout; the caller keeps ownership.
 * Unknown names are ignored (load_state_dict(strict=False)).  Synchronous. */
int wrnn_set_weights(wrnn_t *h, const wrnn_tensor *tensors, int n);

/* Run the whole sample loop (fatchord_version.py:192-241) for B rows × L steps.
 *   cond   [L][B][feat_dims + 4·aux_dims]  upsampled mel ‖ aux, time-major (device);
 *          NULL in DM mode (deepmind_version.generate(seq_len) has no conditioning)
 *   noise  [L][B][K] injected draws in reference order, or NULL for in-kernel Philox:
 *          MOL K = 11 (u1[10], u2 ∈ (1e-5, 1−1e-5), utils/distribution.py:106,118);
 *          RAW K = n_classes (q ~ Exp(1); Categorical.sample ≡ argmax(probs/q));
 *          DM  K = 2·n_classes (q_coarse, then q_fine, deepmind_version.py:130,150)
 *   seed, row_offset  Philox key and global id of row 0 (draws are keyed by
 *          (seed, row_offset + b, step, k), so sharding rows across calls/GPUs is invariant)
 *   out    [B][L] fp32 samples (the values appended at :227/:236; DM: the combined 16-bit
 *          sample coarse·256 + fine − 2^15, utils/dsp.py:33-34)               (device)
 *   labels [B][L] int32 class labels (RAW) / combined samples (DM), or NULL  (device)
 * Asynchronous on `stream`; kernel-side failures surface through wrnn_check. */
int wrnn_generate(wrnn_t *h, const float *cond, int B, int L, const float *noise,
                  uint64_t seed, int64_t row_offset, float *out, int32_t *labels, void *stream);

/* Synchronise `stream` and report a persistent-kernel abort (WRNN_ETIMEOUT) from the
 * last wrnn_generate on it.  The reference raises synchronously; this is that check. */
int wrnn_check(wrnn_t *h, void *stream);

/* Device time (ms, HIP events on the launch stream) from the first to the last persistent
 * loop launch of the last wrnn_generate — the kernel time the roofline is computed from.
 * Waits for that launch to finish. */
int wrnn_elapsed_ms(wrnn_t *h, float *ms);

int wrnn_query(const wrnn_t *h, wrnn_info *info);
const char *wrnn_last_error(const wrnn_t *h);
void wrnn_destroy(wrnn_t *h);

/* ---- conditioning producer and waveform consumer (stateless; no handle) ----------------- */

/* The UpsampleNetwork's mel path: per scale s_i a nearest Stretch2d(s_i) and a Conv2d(1,1,
 * (1, 2·s_i+1), padding (0, s_i), no bias) whose taps are `upsample.up_layers.{2i+1}.weight`
 * (fatchord_version.py:64-79), applied to the mel zero-padded by `pad` frames each side. */
typedef struct {
    int32_t feat_dims;       /* num_mels (80) */
    int32_t res_out_dims;    /* MelResNet output channels (128) = 4·aux_dims */
    int32_t pad;             /* voc_pad (2) */
    int32_t n_scales;        /* 1..4 (hparams voc_upsample_factors = (5, 5, 11)) */
    int32_t scales[4];       /* each 1..15 */
    const float *taps[4];    /* HOST pointers, 2·scales[i]+1 floats each */
} wrnn_upsample_cfg;

/* Shape of the conditioning wrnn_upsample_pack writes for `B` mel rows of `T` frames:
 * steps = L = hop·T unbatched (target <= 0), else the fold window target + 2·overlap;
 * rows = B·num_folds (fold_with_overlap, fatchord_version.py:317-330). */
int wrnn_cond_shape(const wrnn_upsample_cfg *cfg, int B, int T, int target, int overlap,
                    int *steps, int *rows);

/* Replaces, in one kernel, everything between MelResNet and the loop's input
 * (fatchord_version.py:183-205): pad_tensor(pad) → 3× (Stretch2d, Conv2d) → crop indent (:88)
 * for the mel, resnet_stretch (:83) for `aux`, fold_with_overlap (:293-340, target <= 0:
 * unbatched) and the cat/transpose into the time-major records wrnn_generate reads.
 *   mel   [B][feat_dims][T]     the generate() input (device, fp32)
 *   aux   [B][res_out_dims][T]  MelResNet(pad_tensor(mel)) output (device, fp32)
 *   cond  [steps][rows][feat_dims + res_out_dims]  (device; row = b·num_folds + fold) */
int wrnn_upsample_pack(const wrnn_upsample_cfg *cfg, const float *mel, const float *aux, int B, int T,
                       int target, int overlap, float *cond, void *stream);

/* wrnn_upsample_pack + wrnn_generate in one call, from the generate() inputs at FRAME rate
 * (ABI 6): mel [U][feat_dims][T] and aux [U][res_out_dims][T] (MelResNet of the padded mel) for U
 * utterances of T frames each; rows / steps as wrnn_cond_shape (target <= 0: unbatched, row u =
 * utterance u; else utterance u's folds are rows u·nf .. u·nf + nf − 1).  noise, seed, row_offset,
 * out, labels as wrnn_generate.
 * The UpsampleNetwork is linear and frame-shift-invariant, so on the XCD-resident paths the
 * conditioning terms W·[mel_up | aux | 1] are formed as W·(frames) — a GEMM over T frames instead
 * of hop·T samples — plus a per-sample sum of ≤ 8 frame rows weighted by the stretch/conv
 * cascade's response (csrc/frame_terms.hip); the other paths get wrnn_upsample_pack's records.
 * Replaces fatchord_version.py:183-241 (pad → upsample → fold → sample loop). */
int wrnn_generate_frames(wrnn_t *h, const wrnn_upsample_cfg *ucfg, const float *mel, const float *aux, int U, int T,
                         int target, int overlap, const float *noise, uint64_t seed, int64_t row_offset, float *out,
                         int32_t *labels, void *stream);

/* wrnn_generate_frames for the loop rows [row_begin, row_begin + row_count) of that launch only
 * (round-5 addition, same ABI): e.g. a contiguous block of one long utterance's folds on one GPU
 * of a node (wavernn_amd/sharding.py generate_sharded_folds).  The rows keep their
 * place in the utterance (row r = fold r % nf of utterance r / nf); noise [steps][row_count][K],
 * out / labels [row_count][steps]; row_offset keys the Philox draws of launch row j as
 * row_offset + j (pass the global row id of row_begin). */
int wrnn_generate_frames_rows(wrnn_t *h, const wrnn_upsample_cfg *ucfg, const float *mel, const float *aux, int U,
                              int T, int target, int overlap, int row_begin, int row_count, const float *noise,
                              uint64_t seed, int64_t row_offset, float *out, int32_t *labels, void *stream);

/* The frame weights wrnn_generate_frames uses (host, stateless): mel_up(p) = Σ_k coef[φ][k] ·
 * mel[f + k + jlo] for p = f·hop + φ, 0 <= k < nJ — the Stretch2d/Conv2d cascade's response to
 * one frame, float64 rounded to fp32.  coef (nullable) [hop][nJ], coef_cap floats.
 * WRNN_EUNSUPPORTED when pad frames do not cover the response's reach or nJ > 8. */
int wrnn_frame_weights(const wrnn_upsample_cfg *ucfg, int *hop, int *nJ, int *jlo, float *coef, int coef_cap);

/* The UpsampleNetwork's MelResNet (fatchord_version.py:13-48) in inference form, one kernel:
 * conv_in (k = 2·pad + 1) → BN → ReLU → res_blocks × [1×1 conv → BN → ReLU → 1×1 conv → BN →
 * + residual] → conv_out, each BatchNorm (running statistics) folded into its conv on the host.
 *   packed [wrnn_melresnet_floats(cfg)] (device): conv_in W[(c·K + tap)][C] + bias[C], per block
 *          W1[C][C] + b1[C] + W2[C][C] + b2[C], conv_out W[C][R] + bias[R] (k-major matrices)
 *   mel    [U][in_dims][T + 2·pad]  pad_tensor'd mel (device);  aux [U][R][T] (device)
 * WRNN_EUNSUPPORTED for channel counts the kernel's thread layout does not cover. */
typedef struct {
    int32_t in_dims;         /* num_mels (80) */
    int32_t compute_dims;    /* C (128) */
    int32_t res_out_dims;    /* R (128) */
    int32_t res_blocks;      /* 10 */
    int32_t pad;             /* voc_pad (2): conv_in kernel 2·pad + 1 */
} wrnn_melresnet_cfg;
int wrnn_melresnet_floats(const wrnn_melresnet_cfg *cfg);
int wrnn_melresnet(const wrnn_melresnet_cfg *cfg, const float *packed, const float *mel, int U, int T, float *aux,
                   void *stream);
/* The frames per workgroup tile wrnn_melresnet takes for U utterances of T frames on the current
 * device (round-6 addition, same ABI): 16, or 4 when a 16-frame grid has fewer workgroups than the
 * device has CUs (both forms sum every output in the same order: bit-identical); negative WRNN_E*
 * as wrnn_melresnet would return. */
int wrnn_melresnet_tile_frames(const wrnn_melresnet_cfg *cfg, int U, int T);

/* generate()'s float64 post-processing on the device (fatchord_version.py:243-258):
 * decode_mu_law (utils/dsp.py:98-103, mu = n_classes) when `mu_law`, xfade_and_unfold
 * (:342-405) of the `rows` folds when `batched` (else row 0), trim to wave_len, and
 * output[-fade_len:] *= linspace(1, 0, fade_len) (fade_len = 20·hop_length).
 *   y     [rows][steps] fp32 loop output (device);  wave [wave_len] float64 (device)
 * WRNN_EINVAL when fade_len > wave_len (the reference's numpy broadcast error, T < 21). */
int wrnn_postprocess(const float *y, int rows, int steps, int batched, int overlap, int mu_law,
                     int n_classes, int wave_len, int fade_len, double *wave, void *stream);

/* The sampler draws wrnn_generate takes when noise == NULL, materialised (round-6 addition, same
 * ABI): out [steps][rows][K] (device fp32) = draw k of launch row j at step step0 + s, keyed
 * (seed, row_offset + j, step0 + s, k) exactly as every loop kernel keys its in-kernel Philox, so
 * passing `out` as `noise` reproduces the noise == NULL audio.  Philox-4x32-10 (Salmon et al.,
 * SC'11), counter (k >> 2, step, row lo, row hi), key (seed lo, seed hi), word k & 3; the top 24
 * bits m of the word map to
 *   MOL (K = 11: u1[10], u2; utils/distribution.py:106,118): fma(1 − 2e-5, m·2^-24, 1e-5) in fp32,
 *       i.e. U(1e-5, 1 − 1e-5);
 *   RAW (K = n_classes) and DM (K = 2Q: q_coarse then q_fine): −log((m + 1)·2^-24), i.e. Exp(1)
 *       (Categorical.sample ≡ argmax(probs / q), fatchord_version.py:232-235,
 *       deepmind_version.py:130,150).
 * Restated in numpy by oracle/philox.py (tests/test_philox.py, tests/test_gpu_philox.py). */
int wrnn_philox_draws(uint64_t seed, int64_t row_offset, int rows, int step0, int steps, int K, int mode, float *out,
                      void *stream);

/* Message of the last failed stateless call on this thread. */
const char *wrnn_cond_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* WAVERNN_AMD_H */
