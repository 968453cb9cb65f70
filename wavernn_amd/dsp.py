"""Audio helpers on the generation path (the reference's utils/dsp.py subset that generate()
and gen_wavernn.py use).  Feature extraction (STFT/mel, Griffin-Lim) is preprocessing and out
of scope."""
from __future__ import annotations

import math
from pathlib import Path
from typing import Union

import numpy as np


def label_2_float(x, bits):
    """utils/dsp.py:8-9: class label in [0, 2**bits) → [-1, 1]."""
    return 2 * x / (2 ** bits - 1.) - 1.


def float_2_label(x, bits):
    """utils/dsp.py:12-15."""
    assert abs(x).max() <= 1.0
    x = (x + 1.) * (2 ** bits - 1) / 2
    return x.clip(0, 2 ** bits - 1)


def encode_mu_law(x, mu):
    """utils/dsp.py:92-95."""
    mu = mu - 1
    fx = np.sign(x) * np.log(1 + mu * np.abs(x)) / np.log(1 + mu)
    return np.floor((fx + 1) / 2 * mu + 0.5)


def decode_mu_law(y, mu, from_labels=True):
    """utils/dsp.py:98-103 (float64 like the reference's post-processing)."""
    if from_labels:
        y = label_2_float(y, math.log2(mu))
    mu = mu - 1
    return np.sign(y) / mu * ((1 + mu) ** np.abs(y) - 1)


def split_signal(x):
    """utils/dsp.py:26-30: 16-bit → (coarse, fine) 8-bit halves."""
    unsigned = x + 2 ** 15
    return unsigned // 256, unsigned % 256


def combine_signal(coarse, fine):
    """utils/dsp.py:33-34 (deepmind dual-softmax output)."""
    return coarse * 256 + fine - 2 ** 15


def save_wav(x: np.ndarray, path: Union[str, Path, None], sample_rate: int = 22050) -> None:
    """utils/dsp.py:22-23 wrote float32 samples with librosa.output.write_wav (removed in
    librosa >= 0.8); the same IEEE-float WAV is written with scipy.  path None → no file."""
    if path is None:
        return
    from scipy.io import wavfile
    wavfile.write(str(path), int(sample_rate), np.asarray(x, dtype=np.float32))
