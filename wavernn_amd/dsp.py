"""Audio helpers of the reference's utils/dsp.py: everything generate(), gen_wavernn.py and the
training data path touch without librosa (mu-law, labels, 16-bit split, wav I/O, dB scaling,
emphasis filters).  Feature extraction (STFT/mel, Griffin-Lim) is preprocessing and out
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


def load_wav(path: Union[str, Path], sample_rate: int = 22050) -> np.ndarray:
    """utils/dsp.py:18-19 (librosa.load(path, sr)[0]): float32 mono in [-1, 1].  Integer PCM is
    scaled by its full-scale value and channels are averaged, as librosa does; a file at another
    rate raises (librosa's resampler is not in this image, so a resampled result would be
    unpinned)."""
    from scipy.io import wavfile
    sr, x = wavfile.read(str(path))
    if sr != sample_rate:
        raise ValueError(f"{path}: sample rate {sr} != {sample_rate} (resampling not supported)")
    if np.issubdtype(x.dtype, np.integer):
        if x.dtype == np.uint8:
            x = (x.astype(np.float32) - 128.0) / 128.0
        else:
            x = x.astype(np.float32) / float(-np.iinfo(x.dtype).min)
    x = np.asarray(x, dtype=np.float32)
    return x.mean(axis=1, dtype=np.float32) if x.ndim == 2 else x


def encode_16bits(x):
    """utils/dsp.py:37-38."""
    return np.clip(x * 2 ** 15, -2 ** 15, 2 ** 15 - 1).astype(np.int16)


def normalize(S, min_level_db: float = -100):
    """utils/dsp.py:50-51 (min_level_db = hp.min_level_db)."""
    return np.clip((S - min_level_db) / -min_level_db, 0, 1)


def denormalize(S, min_level_db: float = -100):
    """utils/dsp.py:54-55."""
    return (np.clip(S, 0, 1) * -min_level_db) + min_level_db


def amp_to_db(x):
    """utils/dsp.py:58-59."""
    return 20 * np.log10(np.maximum(1e-5, x))


def db_to_amp(x):
    """utils/dsp.py:62-63."""
    return np.power(10.0, x * 0.05)


def pre_emphasis(x, preemphasis: float = 0.97):
    """utils/dsp.py:84-85 (first-order FIR 1 - p·z⁻¹).  The reference reads hp.preemphasis,
    which its hparams.py does not define: callers pass the coefficient."""
    from scipy.signal import lfilter
    return lfilter([1, -preemphasis], [1], x)


def de_emphasis(x, preemphasis: float = 0.97):
    """utils/dsp.py:88-89 (the inverse IIR)."""
    from scipy.signal import lfilter
    return lfilter([1], [1, -preemphasis], x)
