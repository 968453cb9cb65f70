"""Device-side producer and consumer around the sample loop (C-ABI `wrnn_upsample_pack`,
`wrnn_postprocess`, csrc/condition.hip).

* `upsample_pack` turns the generate() mel input and the MelResNet output into the loop's
  time-major conditioning records in one HIP kernel: pad_tensor, the UpsampleNetwork's
  Stretch2d/Conv2d chain and crop, resnet_stretch, fold_with_overlap and the cat/transpose
  (models/fatchord_version.py:82-89, :183-205, :293-340).
* `melresnet` runs the UpsampleNetwork's MelResNet (:13-48) as one HIP kernel on weights packed by
  `melresnet_pack` (every BatchNorm folded into its conv; csrc/melresnet.hip).
* `postprocess` is generate()'s float64 tail on the device: decode_mu_law (utils/dsp.py:98-103),
  xfade_and_unfold (:342-405), trim and the 20·hop linear fade-out (:243-258).

No CPU fallback: the tensors must live on a GPU and the HIP library must be built."""
from __future__ import annotations

import ctypes
from typing import Sequence, Tuple

import numpy as np
import torch

from . import _native as nat


class UpsampleSpec:
    """The mel-path shape of an UpsampleNetwork: scales, taps (host fp32) and pad."""

    def __init__(self, feat_dims: int, res_out_dims: int, pad: int, scales: Sequence[int],
                 taps: Sequence[np.ndarray]):
        if len(scales) != len(taps) or not 1 <= len(scales) <= 4:
            raise ValueError("1..4 upsample scales, one tap vector each")
        self.scales = tuple(int(s) for s in scales)
        self._taps = [np.ascontiguousarray(np.asarray(t, dtype=np.float32).reshape(-1)) for t in taps]
        for s, t in zip(self.scales, self._taps):
            if t.size != 2 * s + 1:
                raise ValueError(f"scale {s} needs {2 * s + 1} taps, got {t.size}")
        self.cfg = nat.UpsampleCfg()
        self.cfg.feat_dims, self.cfg.res_out_dims, self.cfg.pad = feat_dims, res_out_dims, pad
        self.cfg.n_scales = len(self.scales)
        fp = ctypes.POINTER(ctypes.c_float)
        for i, (s, t) in enumerate(zip(self.scales, self._taps)):
            self.cfg.scales[i] = s
            self.cfg.taps[i] = t.ctypes.data_as(fp)
        self.hop = int(np.prod(self.scales))

    @classmethod
    def from_module(cls, upsample, feat_dims: int, pad: int) -> "UpsampleSpec":
        """From an UpsampleNetwork (reference layout: up_layers = [Stretch2d, Conv2d] × n)."""
        convs = [m for m in upsample.up_layers if isinstance(m, torch.nn.Conv2d)]
        scales = [(c.kernel_size[1] - 1) // 2 for c in convs]
        taps = [c.weight.detach().float().cpu().numpy() for c in convs]
        res_out = upsample.resnet.conv_out.out_channels
        return cls(feat_dims, res_out, pad, scales, taps)

    def with_res_out(self, res_out_dims: int) -> "UpsampleSpec":
        """The same cascade for an aux input of res_out_dims channels (zero-padded dims)."""
        return UpsampleSpec(self.cfg.feat_dims, res_out_dims, self.cfg.pad, self.scales, self._taps)

    def shape(self, B: int, T: int, target: int, overlap: int) -> Tuple[int, int]:
        steps, rows = ctypes.c_int(), ctypes.c_int()
        nat.check_cond(nat.lib().wrnn_cond_shape(ctypes.byref(self.cfg), B, T, target, overlap,
                                                 ctypes.byref(steps), ctypes.byref(rows)))
        return steps.value, rows.value


def frame_weights(spec: UpsampleSpec) -> Tuple[int, int, np.ndarray]:
    """(jlo, nJ, coef [hop][nJ]) with mel_up(f·hop + φ) = Σ_k coef[φ][k]·mel[f + k + jlo] — the
    cascade's frame weights wrnn_generate_frames forms the conditioning terms with (host call)."""
    hop, nJ, jlo = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = nat.lib().wrnn_frame_weights(ctypes.byref(spec.cfg), ctypes.byref(hop), ctypes.byref(nJ), ctypes.byref(jlo),
                                      None, 0)
    if rc != 0:
        raise nat.WrnnError(rc, "the upsample cascade has no exact frame-rate form (pad frames < its reach)")
    coef = np.zeros((hop.value, nJ.value), np.float32)
    nat.check_cond(nat.lib().wrnn_frame_weights(ctypes.byref(spec.cfg), None, None, None,
                                                coef.ctypes.data_as(ctypes.c_void_p), coef.size))
    return jlo.value, nJ.value, coef


def melresnet_cfg(resnet) -> "nat.MelResNetCfg":
    """The wrnn_melresnet_cfg of a MelResNet module (reference layout, fatchord_version.py:30-48)."""
    cfg = nat.MelResNetCfg()
    cfg.in_dims = resnet.conv_in.in_channels
    cfg.compute_dims = resnet.conv_in.out_channels
    cfg.res_out_dims = resnet.conv_out.out_channels
    cfg.res_blocks = len(resnet.layers)
    cfg.pad = (resnet.conv_in.kernel_size[0] - 1) // 2
    return cfg


@torch.no_grad()
def melresnet_pack(resnet) -> torch.Tensor:
    """wrnn_melresnet's packed weights from a MelResNet module: each BatchNorm (running statistics,
    eval form) folded into the conv before it — W' = W·γ/√(var + ε), b' = β − μ·γ/√(var + ε), in
    float64 — matrices k-major.  Lives on the module's device."""
    def fold(w, bn):
        s = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
        return w.double() * s.view(-1, *([1] * (w.dim() - 1))), bn.bias.double() - bn.running_mean.double() * s

    parts = []
    w0, b0 = fold(resnet.conv_in.weight, resnet.batch_norm)            # [C][in][K]
    parts += [w0.permute(1, 2, 0).reshape(-1), b0]                     # [(c·K + tap)][C]
    for blk in resnet.layers:
        w1, b1 = fold(blk.conv1.weight[:, :, 0], blk.batch_norm1)
        w2, b2 = fold(blk.conv2.weight[:, :, 0], blk.batch_norm2)
        parts += [w1.t().reshape(-1), b1, w2.t().reshape(-1), b2]
    parts += [resnet.conv_out.weight[:, :, 0].double().t().reshape(-1), resnet.conv_out.bias.double()]
    return torch.cat([p.reshape(-1) for p in parts]).float().contiguous()


def melresnet(cfg, packed: torch.Tensor, mel_padded: torch.Tensor) -> torch.Tensor:
    """MelResNet(pad_tensor(mel)) in one HIP kernel: mel_padded [U][in][T + 2·pad] → aux [U][R][T].
    Raises WrnnError(WRNN_EUNSUPPORTED) for channel counts the kernel does not cover."""
    _need_gpu(mel_padded, packed)
    x = mel_padded.contiguous().float()
    U, cin, Tp = x.shape
    T = Tp - 2 * cfg.pad
    if cin != cfg.in_dims or T < 1 or packed.numel() != nat.lib().wrnn_melresnet_floats(ctypes.byref(cfg)):
        raise ValueError("mel / packed weights do not match the MelResNet config")
    aux = torch.empty(U, cfg.res_out_dims, T, device=x.device, dtype=torch.float32)
    rc = nat.lib().wrnn_melresnet(ctypes.byref(cfg), packed.data_ptr(), x.data_ptr(), U, T, aux.data_ptr(),
                                  _stream(x.device))
    if rc != 0:
        raise nat.WrnnError(rc, "wrnn_melresnet")
    return aux


def _stream(dev: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _need_gpu(*ts: torch.Tensor) -> None:
    for t in ts:
        if t.device.type != "cuda":
            raise RuntimeError("the conditioning/post-processing kernels run on the MI355X: tensors must be on a "
                               "GPU (no CPU fallback)")


def upsample_pack(spec: UpsampleSpec, mel: torch.Tensor, aux: torch.Tensor, target: int = 0,
                  overlap: int = 0) -> torch.Tensor:
    """mel [B][feat][T], aux [B][res_out][T] (MelResNet of the padded mel) → cond
    [steps][rows][feat + res_out] fp32; target <= 0 means unbatched."""
    _need_gpu(mel, aux)
    mel = mel.contiguous().float()
    aux = aux.contiguous().float()
    B, feat, T = mel.shape
    if feat != spec.cfg.feat_dims or aux.shape != (B, spec.cfg.res_out_dims, T):
        raise ValueError(f"mel {tuple(mel.shape)} / aux {tuple(aux.shape)} do not match the upsample spec")
    steps, rows = spec.shape(B, T, target, overlap)
    cond = torch.empty(steps, rows, feat + spec.cfg.res_out_dims, device=mel.device, dtype=torch.float32)
    nat.check_cond(nat.lib().wrnn_upsample_pack(ctypes.byref(spec.cfg), mel.data_ptr(), aux.data_ptr(), B, T,
                                                target, overlap, cond.data_ptr(), _stream(mel.device)))
    return cond


def postprocess(y: torch.Tensor, batched: bool, overlap: int, mu_law: bool, n_classes: int, wave_len: int,
                fade_len: int) -> torch.Tensor:
    """Loop output y [rows][steps] fp32 → float64 waveform [wave_len] (device tensor)."""
    _need_gpu(y)
    y = y.contiguous().float()
    rows, steps = y.shape
    if fade_len > wave_len:
        # the reference fails here in numpy (output[-fade:] *= fade_out, :255-258)
        raise ValueError(f"operands could not be broadcast together with shapes ({wave_len},) ({fade_len},) ")
    wave = torch.empty(wave_len, device=y.device, dtype=torch.float64)
    nat.check_cond(nat.lib().wrnn_postprocess(y.data_ptr(), rows, steps, int(batched), overlap, int(mu_law),
                                              n_classes, wave_len, fade_len, wave.data_ptr(), _stream(y.device)))
    return wave
