"""Deterministic synthetic inputs for the WaveRNN generation path.

There are no pretrained weights (the reference's `pretrained/*.zip` are absent,
SURVEY.md §8(c)), so every configuration runs on random weights.  This module is
the single documented generator used by the golden-fixture script, the tests and
`bench.py`; the fixtures store a SHA-256 of what it produced so any drift in it is
caught instead of silently invalidating the goldens.

Key naming and shapes follow the reference state_dict of
`models/fatchord_version.py:92-129` (measured key list: SURVEY.md §8(a15)) and
`models/deepmind_version.py:9-34`.
"""
from __future__ import annotations

import hashlib
import zlib
from dataclasses import dataclass, field
from typing import Dict, Tuple

import numpy as np


@dataclass(frozen=True)
class FatchordDims:
    """Constructor arguments of the reference `WaveRNN` (fatchord_version.py:93-95)."""
    rnn_dims: int = 512
    fc_dims: int = 512
    bits: int = 9
    pad: int = 2
    upsample_factors: Tuple[int, ...] = (5, 5, 11)
    feat_dims: int = 80
    compute_dims: int = 128
    res_out_dims: int = 128
    res_blocks: int = 10
    hop_length: int = 275
    sample_rate: int = 22050
    mode: str = "MOL"

    @property
    def aux_dims(self) -> int:          # fatchord_version.py:110
        return self.res_out_dims // 4

    @property
    def n_classes(self) -> int:         # fatchord_version.py:99-102
        return 2 ** self.bits if self.mode == "RAW" else 30

    def ctor_kwargs(self) -> dict:
        return dict(rnn_dims=self.rnn_dims, fc_dims=self.fc_dims, bits=self.bits, pad=self.pad,
                    upsample_factors=self.upsample_factors, feat_dims=self.feat_dims,
                    compute_dims=self.compute_dims, res_out_dims=self.res_out_dims,
                    res_blocks=self.res_blocks, hop_length=self.hop_length,
                    sample_rate=self.sample_rate, mode=self.mode)


# The hparams.py vocoder section (hparams.py:20-44) in the 800k MoL configuration.
DEFAULT_MOL = FatchordDims()
DEFAULT_RAW = FatchordDims(mode="RAW")
# Small dims used to exercise the generic-dimension code paths (fc != rnn, bits != 9).
TINY_RAW = FatchordDims(rnn_dims=64, fc_dims=96, bits=8, compute_dims=16, res_out_dims=16,
                        res_blocks=1, mode="RAW")
TINY_MOL = FatchordDims(rnn_dims=64, fc_dims=96, compute_dims=16, res_out_dims=16,
                        res_blocks=1, mode="MOL")
# BASELINE config 4: rnn_dims 896 with 4x4 block-sparse GRU weights (pruning.prune_state, 95 %)
SPARSE896_MOL = FatchordDims(rnn_dims=896, mode="MOL")


def fatchord_state_shapes(d: FatchordDims) -> Dict[str, Tuple[tuple, str]]:
    """Every state_dict key of the reference model → (shape, kind)."""
    s: Dict[str, Tuple[tuple, str]] = {"step": ((1,), "step")}
    c, k = d.compute_dims, 2 * d.pad + 1
    s["upsample.resnet.conv_in.weight"] = ((c, d.feat_dims, k), "w")

    def bn(prefix: str):
        s[prefix + ".weight"] = ((c,), "bn_w")
        s[prefix + ".bias"] = ((c,), "bn_b")
        s[prefix + ".running_mean"] = ((c,), "bn_rm")
        s[prefix + ".running_var"] = ((c,), "bn_rv")
        s[prefix + ".num_batches_tracked"] = ((), "nbt")

    bn("upsample.resnet.batch_norm")
    for i in range(d.res_blocks):
        p = f"upsample.resnet.layers.{i}"
        s[p + ".conv1.weight"] = ((c, c, 1), "w")
        s[p + ".conv2.weight"] = ((c, c, 1), "w")
        bn(p + ".batch_norm1")
        bn(p + ".batch_norm2")
    s["upsample.resnet.conv_out.weight"] = ((d.res_out_dims, c, 1), "w")
    s["upsample.resnet.conv_out.bias"] = ((d.res_out_dims,), "b:upsample.resnet.conv_out.weight")
    for i, sc in enumerate(d.upsample_factors):
        s[f"upsample.up_layers.{2 * i + 1}.weight"] = ((1, 1, 1, 2 * sc + 1), "box")
    r, f, a = d.rnn_dims, d.fc_dims, d.aux_dims
    s["I.weight"] = ((r, d.feat_dims + a + 1), "w")
    s["I.bias"] = ((r,), "b:I.weight")
    for name, n_in in (("rnn1", r), ("rnn2", r + a)):
        s[f"{name}.weight_ih_l0"] = ((3 * r, n_in), "w")
        s[f"{name}.weight_hh_l0"] = ((3 * r, r), "w")
        s[f"{name}.bias_ih_l0"] = ((3 * r,), f"b:{name}.weight_ih_l0")
        s[f"{name}.bias_hh_l0"] = ((3 * r,), f"b:{name}.weight_hh_l0")
    s["fc1.weight"] = ((f, r + a), "w")
    s["fc1.bias"] = ((f,), "b:fc1.weight")
    s["fc2.weight"] = ((f, f + a), "w")
    s["fc2.bias"] = ((f,), "b:fc2.weight")
    s["fc3.weight"] = ((d.n_classes, f), "w")
    s["fc3.bias"] = ((d.n_classes,), "b:fc3.weight")
    return s


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.default_rng(np.random.SeedSequence([seed, zlib.crc32(key.encode())]))


def make_fatchord_state(d: FatchordDims, seed: int = 0, step: int = 800_000) -> Dict[str, np.ndarray]:
    """Random weights in the reference layout: weights/biases U(±1/sqrt(fan_in)) as torch's
    default init, BatchNorm statistics in a plausible range, up-layer box filters 1/k (the
    reference's init, fatchord_version.py:78) with ±10% jitter.  One independent stream per key."""
    shapes = fatchord_state_shapes(d)
    out: Dict[str, np.ndarray] = {}
    for key in sorted(shapes):
        shape, kind = shapes[key]
        g = _rng(seed, key)
        if kind == "step":
            out[key] = np.array([step], dtype=np.int64)
        elif kind == "nbt":
            out[key] = np.array(0, dtype=np.int64)
        elif kind == "w":
            bound = 1.0 / np.sqrt(float(np.prod(shape[1:])))
            out[key] = g.uniform(-bound, bound, size=shape).astype(np.float32)
        elif kind.startswith("b:"):
            wshape = shapes[kind[2:]][0]
            bound = 1.0 / np.sqrt(float(np.prod(wshape[1:])))
            out[key] = g.uniform(-bound, bound, size=shape).astype(np.float32)
        elif kind == "bn_w":
            out[key] = g.uniform(0.8, 1.2, size=shape).astype(np.float32)
        elif kind == "bn_b":
            out[key] = g.uniform(-0.1, 0.1, size=shape).astype(np.float32)
        elif kind == "bn_rm":
            out[key] = g.uniform(-0.2, 0.2, size=shape).astype(np.float32)
        elif kind == "bn_rv":
            out[key] = g.uniform(0.5, 1.5, size=shape).astype(np.float32)
        elif kind == "box":
            kk = shape[-1]
            out[key] = (np.full(shape, 1.0 / kk) * (1.0 + g.uniform(-0.1, 0.1, size=shape))).astype(np.float32)
        else:  # pragma: no cover
            raise ValueError(kind)
    # Shape the output head like a trained vocoder's so parity tests are sensitive to the
    # network arithmetic: with plain init the RAW softmax is ~uniform (labels then follow
    # the Exp(1) noise alone) and MoL log-scales ~0 clamp half the samples to ±1.
    if d.mode == "RAW":
        out["fc3.weight"] = (out["fc3.weight"] * np.float32(16.0)).astype(np.float32)
    else:
        nr = d.n_classes // 3
        out["fc3.bias"][2 * nr:] -= np.float32(5.0)
    return out


def make_mel(n_mels: int, n_frames: int, seed: int = 1) -> np.ndarray:
    """Normalised mel (n_mels, T) in [0, 1) — the range gen_wavernn.py:52-55 accepts."""
    return np.random.default_rng(seed).random((n_mels, n_frames), dtype=np.float32)


def frames_for_seconds(seconds: float, sample_rate: int = 22050, hop: int = 275) -> int:
    """T such that wave_len = hop*(T-1) covers `seconds`."""
    return int(seconds * sample_rate / hop) + 1


def make_conditioning(B: int, L: int, feat: int, res_out: int, seed: int = 2):
    """Upsampled conditioning as generate() sees it after fold: mels [B][L][feat] in [0,1),
    aux [B][L][res_out] ~ 0.5·N(0,1) (MelResNet output scale)."""
    g = np.random.default_rng(seed)
    mels = g.random((B, L, feat), dtype=np.float32)
    aux = (0.5 * g.standard_normal((B, L, res_out))).astype(np.float32)
    return mels, aux


MOL_NOISE_K = 11   # u1[10] (mixture Gumbel draw) then u2 (logistic draw): distribution.py:106,118


def make_noise(mode: str, B: int, L: int, n_classes: int, seed: int = 3) -> np.ndarray:
    """Injected noise in the reference draw order, layout [L][B][K].

    MOL: u1[0:10] then u2, both U(1e-5, 1-1e-5) (utils/distribution.py:106,118).
    RAW: q[0:n_classes] ~ Exp(1); Categorical.sample() ≡ argmax(probs / q).
    """
    g = np.random.default_rng(seed)
    if mode == "MOL":
        u = g.random((L, B, MOL_NOISE_K))
        u = 1e-5 + (1.0 - 2e-5) * u
        return np.clip(u.astype(np.float32), np.float32(1e-5), np.float32(1.0 - 1e-5))
    if mode == "RAW":
        q = g.standard_exponential((L, B, n_classes), dtype=np.float32)
        return np.maximum(q, np.float32(1e-30))
    raise ValueError(mode)


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def state_digest(state: Dict[str, np.ndarray]) -> str:
    return digest(*[state[k] for k in sorted(state)])


# ---------------------------------------------------------------------- deepmind_version
@dataclass(frozen=True)
class DeepmindDims:
    """Constructor arguments of models/deepmind_version.py:WaveRNN (:9-34)."""
    hidden_size: int = 896
    quantisation: int = 256

    @property
    def split_size(self) -> int:
        return self.hidden_size // 2

    def ctor_kwargs(self) -> dict:
        return dict(hidden_size=self.hidden_size, quantisation=self.quantisation)


DEFAULT_DM = DeepmindDims()
TINY_DM = DeepmindDims(hidden_size=64, quantisation=256)


def deepmind_state_shapes(d: DeepmindDims) -> Dict[str, tuple]:
    H, S, Q = d.hidden_size, d.split_size, d.quantisation
    return {"R.weight": (3 * H, H), "O1.weight": (S, S), "O1.bias": (S,), "O2.weight": (Q, S), "O2.bias": (Q,),
            "O3.weight": (S, S), "O3.bias": (S,), "O4.weight": (Q, S), "O4.bias": (Q,),
            "I_coarse.weight": (3 * S, 2), "I_fine.weight": (3 * S, 3),
            "bias_u": (H,), "bias_r": (H,), "bias_e": (H,)}


def make_deepmind_state(d: DeepmindDims, seed: int = 0) -> Dict[str, np.ndarray]:
    """Random weights U(±1/sqrt(fan_in)) (torch Linear init); the gate biases (zeros in the
    reference init, :29-31) get U(±0.1) and the two output heads are scaled ×16, so the sampled
    labels depend on the network arithmetic and not only on the noise."""
    out: Dict[str, np.ndarray] = {}
    for key, shape in sorted(deepmind_state_shapes(d).items()):
        g = _rng(seed, "dm:" + key)
        if key.startswith("bias_"):
            out[key] = g.uniform(-0.1, 0.1, size=shape).astype(np.float32)
            continue
        fan_in = shape[1] if len(shape) == 2 else deepmind_state_shapes(d)[key.replace("bias", "weight")][1]
        bound = 1.0 / np.sqrt(float(fan_in))
        out[key] = g.uniform(-bound, bound, size=shape).astype(np.float32)
    for k in ("O2.weight", "O4.weight"):
        out[k] = (out[k] * np.float32(16.0)).astype(np.float32)
    return out


def make_dm_noise(B: int, L: int, Q: int = 256, seed: int = 3) -> np.ndarray:
    """Exp(1) draws [L][B][2·Q]: the coarse Categorical's q, then the fine one's, per step."""
    g = np.random.default_rng(seed)
    return g.exponential(1.0, size=(L, B, 2 * Q)).astype(np.float32)
