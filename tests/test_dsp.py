"""utils/dsp.py helpers (dsp.py:8-103) restated in wavernn_amd.dsp: closed-form checks and
round trips (librosa is absent here, so wav I/O is checked against its documented scaling)."""
import numpy as np
import pytest

from wavernn_amd import dsp


def test_db_and_normalize_round_trip():
    x = np.linspace(1e-4, 3.0, 50)
    np.testing.assert_allclose(dsp.db_to_amp(dsp.amp_to_db(x)), x, rtol=1e-12)
    assert dsp.amp_to_db(np.array([0.0]))[0] == pytest.approx(-100.0)
    S = np.linspace(-100, 0, 11)
    np.testing.assert_allclose(dsp.normalize(S), np.linspace(0, 1, 11), atol=1e-15)
    np.testing.assert_allclose(dsp.denormalize(dsp.normalize(S)), S, atol=1e-12)
    assert dsp.normalize(np.array([-150.0, 20.0])).tolist() == [0.0, 1.0]


def test_emphasis_inverse_and_16bits():
    g = np.random.default_rng(0)
    x = g.uniform(-1, 1, 1000)
    y = dsp.pre_emphasis(x)
    assert y[0] == x[0] and y[5] == pytest.approx(x[5] - 0.97 * x[4])
    np.testing.assert_allclose(dsp.de_emphasis(y), x, atol=1e-12)
    e = dsp.encode_16bits(np.array([-1.5, -1.0, 0.0, 0.5, 1.0]))
    assert e.dtype == np.int16 and e.tolist() == [-32768, -32768, 0, 16384, 32767]
    c, f = dsp.split_signal(e.astype(np.int64))
    assert dsp.combine_signal(c, f).tolist() == e.tolist()


def test_wav_round_trip(tmp_path):
    x = np.random.default_rng(1).uniform(-1, 1, 2000).astype(np.float32)
    p = tmp_path / "a.wav"
    dsp.save_wav(x, p, 22050)
    np.testing.assert_array_equal(dsp.load_wav(p, 22050), x)
    from scipy.io import wavfile
    pcm = np.stack([dsp.encode_16bits(x), dsp.encode_16bits(-x)], 1)
    wavfile.write(str(tmp_path / "b.wav"), 22050, pcm)
    y = dsp.load_wav(tmp_path / "b.wav", 22050)
    assert y.dtype == np.float32 and y.shape == (2000,)
    np.testing.assert_allclose(y, (pcm[:, 0] / 32768.0 + pcm[:, 1] / 32768.0) / 2, atol=1e-7)
    with pytest.raises(ValueError):
        dsp.load_wav(p, 16000)


def test_wav_integer_pcm_scaling(tmp_path):
    """uint8 PCM → (x − 128) / 128; int32 (and 24-bit, which scipy reads left-justified into
    int32) → x / 2**31: librosa's full-scale conventions."""
    from scipy.io import wavfile
    u8 = np.array([0, 1, 64, 128, 200, 255], dtype=np.uint8)
    wavfile.write(str(tmp_path / "u8.wav"), 22050, u8)
    y = dsp.load_wav(tmp_path / "u8.wav", 22050)
    assert y.dtype == np.float32
    np.testing.assert_array_equal(y, (u8.astype(np.float32) - 128.0) / 128.0)
    i32 = np.array([-2 ** 31, -1, 0, 1, 2 ** 30, 2 ** 31 - 1], dtype=np.int32)
    wavfile.write(str(tmp_path / "i32.wav"), 22050, i32)
    y = dsp.load_wav(tmp_path / "i32.wav", 22050)
    np.testing.assert_array_equal(y, i32.astype(np.float32) / np.float32(2 ** 31))
    assert y.min() == -1.0 and y.max() <= 1.0
