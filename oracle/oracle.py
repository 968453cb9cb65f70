"""Oracle: CPU restatement of the reference WaveRNN generation path.

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package `wavernn_amd` (which must fail loudly
when its HIP library is missing instead of falling back here).

Pinned against tests/golden/*.npz (outputs of the reference generate() itself, made by
tests/golden/make_golden.py) in tests/test_oracle_golden.py.

  loop (C, oracle/wavernn_oracle.c)   fatchord_version.py:201-237, distribution.py:87-123,
                                      deepmind_version.py:75-165
  upsample (numpy, below)             fatchord_version.py:13-89
  pad / fold / xfade / fade (numpy)   fatchord_version.py:183-190, 243-258, 281-405
  mu-law decode (numpy)               utils/dsp.py:8-9, 98-103
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from typing import Dict, Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

_F = ctypes.POINTER(ctypes.c_float)
_I32 = ctypes.POINTER(ctypes.c_int32)


class _Dims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("rnn", "fc", "aux", "feat", "n_classes", "mol")]


class _Weights(ctypes.Structure):
    _fields_ = [(n, _F) for n in (
        "I_w", "I_b", "rnn1_wih", "rnn1_whh", "rnn1_bih", "rnn1_bhh",
        "rnn2_wih", "rnn2_whh", "rnn2_bih", "rnn2_bhh",
        "fc1_w", "fc1_b", "fc2_w", "fc2_b", "fc3_w", "fc3_b")]


class _DMWeights(ctypes.Structure):
    _fields_ = [(n, _F) for n in (
        "R", "O1_w", "O1_b", "O2_w", "O2_b", "O3_w", "O3_b", "O4_w", "O4_b",
        "Ic", "If", "bu", "br", "be")]


_FATCHORD_KEYS = {
    "I_w": "I.weight", "I_b": "I.bias",
    "rnn1_wih": "rnn1.weight_ih_l0", "rnn1_whh": "rnn1.weight_hh_l0",
    "rnn1_bih": "rnn1.bias_ih_l0", "rnn1_bhh": "rnn1.bias_hh_l0",
    "rnn2_wih": "rnn2.weight_ih_l0", "rnn2_whh": "rnn2.weight_hh_l0",
    "rnn2_bih": "rnn2.bias_ih_l0", "rnn2_bhh": "rnn2.bias_hh_l0",
    "fc1_w": "fc1.weight", "fc1_b": "fc1.bias", "fc2_w": "fc2.weight", "fc2_b": "fc2.bias",
    "fc3_w": "fc3.weight", "fc3_b": "fc3.bias",
}

_DM_KEYS = {
    "R": "R.weight", "O1_w": "O1.weight", "O1_b": "O1.bias", "O2_w": "O2.weight", "O2_b": "O2.bias",
    "O3_w": "O3.weight", "O3_b": "O3.bias", "O4_w": "O4.weight", "O4_b": "O4.bias",
    "Ic": "I_coarse.weight", "If": "I_fine.weight", "bu": "bias_u", "br": "bias_r", "be": "bias_e",
}


def build(verbose: bool = False) -> str:
    """Compile the C restatement (gcc, no GPU toolchain involved)."""
    os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
    src = os.path.join(HERE, "wavernn_oracle.c")
    if os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= os.path.getmtime(src):
        return LIB_PATH
    cmd = ["gcc", "-O3", "-fPIC", "-shared", "-fno-fast-math", "-o", LIB_PATH, src, "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.orc_fatchord_loop.restype = ctypes.c_int
        _lib.orc_fatchord_loop.argtypes = [ctypes.POINTER(_Dims), ctypes.POINTER(_Weights), _F, _F,
                                           ctypes.c_int, ctypes.c_int, _F, _F, _I32]
        _lib.orc_deepmind_loop.restype = ctypes.c_int
        _lib.orc_deepmind_loop.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_DMWeights),
                                           ctypes.c_int, ctypes.c_int, _F, _I32, _I32]
    return _lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_F)


def fatchord_loop(state: Dict[str, np.ndarray], mode: str, mels: np.ndarray, aux: np.ndarray,
                  noise: np.ndarray) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """Run the reference loop (fatchord_version.py:201-237) on folded conditioning.

    mels [B][L][feat], aux [B][L][4·aux_dims], noise [L][B][K] → (samples [B][L] f32,
    labels [B][L] int32 or None)."""
    mels = np.ascontiguousarray(mels, dtype=np.float32)
    aux = np.ascontiguousarray(aux, dtype=np.float32)
    noise = np.ascontiguousarray(noise, dtype=np.float32)
    B, L, feat = mels.shape
    rnn = state["I.weight"].shape[0]
    a = aux.shape[2] // 4
    fc = state["fc1.weight"].shape[0]
    nc = state["fc3.weight"].shape[0]
    mol = 1 if mode == "MOL" else 0
    assert noise.shape == (L, B, 11 if mol else nc), noise.shape
    ws = {f: np.ascontiguousarray(state[k], dtype=np.float32) for f, k in _FATCHORD_KEYS.items()}
    w = _Weights(**{f: _fp(v) for f, v in ws.items()})
    d = _Dims(rnn, fc, a, feat, nc, mol)
    out = np.zeros((B, L), np.float32)
    labels = None if mol else np.zeros((B, L), np.int32)
    rc = lib().orc_fatchord_loop(ctypes.byref(d), ctypes.byref(w), _fp(mels), _fp(aux), B, L,
                                 _fp(noise), _fp(out),
                                 labels.ctypes.data_as(_I32) if labels is not None else None)
    if rc != 0:
        raise MemoryError("oracle allocation failed")
    return out, labels


def deepmind_loop(state: Dict[str, np.ndarray], B: int, L: int, noise: np.ndarray):
    """deepmind_version.py:75-165 for B independent rows; noise [L][B][2·Q].
    Returns (coarse, fine, output) with output = coarse·256 + fine − 2¹⁵ (utils/dsp.py:33-34)."""
    H = state["R.weight"].shape[1]
    Q = state["O2.weight"].shape[0]
    noise = np.ascontiguousarray(noise, dtype=np.float32)
    assert noise.shape == (L, B, 2 * Q)
    ws = {f: np.ascontiguousarray(state[k], dtype=np.float32) for f, k in _DM_KEYS.items()}
    w = _DMWeights(**{f: _fp(v) for f, v in ws.items()})
    coarse = np.zeros((B, L), np.int32)
    fine = np.zeros((B, L), np.int32)
    rc = lib().orc_deepmind_loop(H, Q, ctypes.byref(w), B, L, _fp(noise),
                                 coarse.ctypes.data_as(_I32), fine.ctypes.data_as(_I32))
    if rc != 0:
        raise MemoryError("oracle allocation failed")
    return coarse, fine, coarse.astype(np.int64) * 256 + fine - 2 ** 15


# ------------------------------------------------------------------- numpy pre-processing
def _bn(x, state, p, eps=1e-5):
    """BatchNorm1d in eval mode (running statistics)."""
    w, b = state[p + ".weight"], state[p + ".bias"]
    rm, rv = state[p + ".running_mean"], state[p + ".running_var"]
    return ((x - rm[:, None]) / np.sqrt(rv[:, None] + eps)) * w[:, None] + b[:, None]


def _conv1x1(w, x):
    return w[:, :, 0] @ x


def melresnet(x: np.ndarray, state, res_blocks: int) -> np.ndarray:
    """MelResNet.forward (fatchord_version.py:31-48); x [feat][T+2pad] → [res_out][T]."""
    w = state["upsample.resnet.conv_in.weight"]          # [C][feat][k]
    k = w.shape[2]
    T = x.shape[1] - k + 1
    y = np.zeros((w.shape[0], T), np.float64)
    for j in range(k):
        y += w[:, :, j].astype(np.float64) @ x[:, j:j + T].astype(np.float64)
    y = np.maximum(_bn(y, state, "upsample.resnet.batch_norm"), 0)
    for i in range(res_blocks):                           # ResBlock (:13-28)
        p = f"upsample.resnet.layers.{i}"
        r = y
        y = np.maximum(_bn(_conv1x1(state[p + ".conv1.weight"], y), state, p + ".batch_norm1"), 0)
        y = _bn(_conv1x1(state[p + ".conv2.weight"], y), state, p + ".batch_norm2") + r
    return _conv1x1(state["upsample.resnet.conv_out.weight"], y) + state["upsample.resnet.conv_out.bias"][:, None]


def upsample(mel_padded: np.ndarray, state, upsample_factors, res_blocks: int, pad: int):
    """UpsampleNetwork.forward (fatchord_version.py:82-89).
    mel_padded [feat][T+2pad] → (mels [L][feat], aux [L][res_out]), L = hop·T."""
    total = int(np.prod(upsample_factors))
    aux = np.repeat(melresnet(mel_padded, state, res_blocks), total, axis=1)   # Stretch2d(total, 1)
    m = mel_padded.astype(np.float64)
    for i, s in enumerate(upsample_factors):
        m = np.repeat(m, s, axis=1)                                            # Stretch2d(s, 1)
        kern = state[f"upsample.up_layers.{2 * i + 1}.weight"].reshape(-1).astype(np.float64)
        mp = np.pad(m, ((0, 0), (s, s)))                                       # Conv2d pad (0, s)
        m = sum(kern[j] * mp[:, j:j + m.shape[1]] for j in range(2 * s + 1))
    indent = pad * total
    m = m[:, indent:-indent]
    return m.T.astype(np.float32), aux.T.astype(np.float32)


def pad_tensor(x: np.ndarray, pad: int, side: str = "both") -> np.ndarray:
    """fatchord_version.py:281-291 on [b][t][c]."""
    b, t, c = x.shape
    total = t + 2 * pad if side == "both" else t + pad
    out = np.zeros((b, total, c), np.float32)
    if side in ("before", "both"):
        out[:, pad:pad + t] = x
    else:
        out[:, :t] = x
    return out


def fold_with_overlap(x: np.ndarray, target: int, overlap: int) -> np.ndarray:
    """fatchord_version.py:293-340; x [1][L][F] → [num_folds][target+2·overlap][F]."""
    _, total_len, features = x.shape
    num_folds = (total_len - overlap) // (target + overlap)
    extended_len = num_folds * (overlap + target) + overlap
    remaining = total_len - extended_len
    if remaining != 0:
        num_folds += 1
        x = pad_tensor(x, target + 2 * overlap - remaining, side="after")
    folded = np.zeros((num_folds, target + 2 * overlap, features), np.float32)
    for i in range(num_folds):
        start = i * (target + overlap)
        folded[i] = x[0, start:start + target + 2 * overlap]
    return folded


def xfade_and_unfold(y: np.ndarray, overlap: int) -> np.ndarray:
    """fatchord_version.py:342-405 (float64; fade_out is prefixed with ones, :382,391)."""
    y = y.copy()
    num_folds, length = y.shape
    target = length - 2 * overlap
    total_len = num_folds * (target + overlap) + overlap
    silence_len = overlap // 2
    fade_len = overlap - silence_len
    t = np.linspace(-1, 1, fade_len, dtype=np.float64)
    fade_in = np.concatenate([np.zeros(silence_len), np.sqrt(0.5 * (1 + t))])
    fade_out = np.concatenate([np.ones(silence_len), np.sqrt(0.5 * (1 - t))])
    y[:, :overlap] *= fade_in
    y[:, -overlap:] *= fade_out
    unfolded = np.zeros(total_len, np.float64)
    for i in range(num_folds):
        start = i * (target + overlap)
        unfolded[start:start + target + 2 * overlap] += y[i]
    return unfolded


def decode_mu_law(y: np.ndarray, mu: int, from_labels: bool = True) -> np.ndarray:
    """utils/dsp.py:98-103 (label_2_float :8-9 when from_labels)."""
    if from_labels:
        bits = math.log2(mu)
        y = 2 * y / (2 ** bits - 1.) - 1.
    mu = mu - 1
    return np.sign(y) / mu * ((1 + mu) ** np.abs(y) - 1)


def generate(state, dims, mel: np.ndarray, batched: bool, target: int, overlap: int, mu_law: bool,
             noise: np.ndarray) -> np.ndarray:
    """Whole WaveRNN.generate (fatchord_version.py:169-264) minus the wav write.
    `dims` is a wavernn_amd.synthetic.FatchordDims-like object; noise [Lf][B][K]."""
    mu_law = mu_law if dims.mode == "RAW" else False                          # (:174)
    T = mel.shape[-1]
    wave_len = (T - 1) * dims.hop_length                                       # (:184)
    mp = pad_tensor(mel.T[None].astype(np.float32), dims.pad)[0].T             # (:185)
    m, a = upsample(mp, state, dims.upsample_factors, dims.res_blocks, dims.pad)
    m, a = m[None], a[None]
    if batched:                                                                # (:188-190)
        m = fold_with_overlap(m, target, overlap)
        a = fold_with_overlap(a, target, overlap)
    out, _ = fatchord_loop(state, dims.mode, m, a, noise)
    return postprocess(out, batched, overlap, mu_law, dims.n_classes, wave_len, 20 * dims.hop_length)


def postprocess(out: np.ndarray, batched: bool, overlap: int, mu_law: bool, n_classes: int, wave_len: int,
                fade_len: int) -> np.ndarray:
    """generate()'s float64 tail (fatchord_version.py:243-258) on the loop output [B][L]."""
    out = out.astype(np.float64)                                               # (:243-245)
    if mu_law:
        out = decode_mu_law(out, n_classes, False)                             # (:247-248)
    out = xfade_and_unfold(out, overlap) if batched else out[0]                # (:250-253)
    fade_out = np.linspace(1, 0, fade_len)                                     # (:256-258)
    out = out[:wave_len]
    out[-fade_len:] *= fade_out
    return out
