"""CLI input validation (gen_wavernn.py:48-57 semantics) and the hparams pseudo-module."""
import numpy as np
import pytest

from wavernn_amd.gen_wavernn import load_mel
from wavernn_amd.hparams import DEFAULTS, HParams


def test_load_mel_checks_shape_and_range(tmp_path):
    good = tmp_path / "m.npy"
    np.save(good, np.random.default_rng(0).random((80, 30)).astype(np.float32))
    assert load_mel(good, 80).shape == (80, 30)
    bad = tmp_path / "b.npy"
    np.save(bad, np.full((80, 30), 2.0, np.float32))
    with pytest.raises(ValueError, match="range"):
        load_mel(bad, 80)
    with pytest.raises(ValueError, match="n_mels"):
        load_mel(good, 64)
    with pytest.raises(ValueError, match=".npy"):
        load_mel(tmp_path / "x.wav", 80)


def test_hparams_configure_once(tmp_path):
    f = tmp_path / "hp.py"
    f.write_text("voc_rnn_dims = 896\nvoc_mode = 'RAW'\n")
    hp = HParams()
    with pytest.raises(AttributeError):
        _ = hp.voc_rnn_dims
    hp.configure(f)
    assert hp.voc_rnn_dims == 896 and hp.voc_mode == "RAW" and hp.hop_length == DEFAULTS["hop_length"]
    with pytest.raises(RuntimeError):
        hp.configure(f)
