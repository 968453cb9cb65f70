"""TTS caller (gen_tacotron.py:142-168 on the MI355X vocoder): the Tacotron → vocoder rescale,
output naming, and the call sequence; on the GPU, synthesize() through the real drop-in."""
import numpy as np
import pytest
import torch

from wavernn_amd.gen_tacotron import _SavedMels, output_name, synthesize, tacotron_mel_to_vocoder, vocoder_type


class _FakeTacotron:
    def __init__(self, mels):
        self.mels = mels
        self.seen = []

    def generate(self, x):
        self.seen.append(x)
        return None, self.mels[x], f"attn{x}"


class _RecordingVocoder:
    def __init__(self):
        self.calls = []

    def generate(self, mels, save_path, batched, target, overlap, mu_law, *, seed=None):
        self.calls.append((mels.clone(), save_path, batched, target, overlap, mu_law, seed))
        return np.zeros(4)


def test_rescale_matches_reference_formula():
    rng = np.random.default_rng(0)
    m = (rng.standard_normal((80, 37)) * 5).astype(np.float32)     # spills past [-4, 4]
    ref = (m + 4) / 8                                               # gen_tacotron.py:147-148
    np.clip(ref, 0, 1, out=ref)
    out = tacotron_mel_to_vocoder(m.copy())
    assert out.shape == (1, 80, 37) and out.dtype == torch.float32
    assert np.array_equal(out[0].numpy(), ref)
    assert out.min() >= 0 and out.max() <= 1


def test_output_names_follow_reference():
    assert vocoder_type(True) == "wavernn_batched" and vocoder_type(False) == "wavernn_unbatched"
    assert output_name(3, "wavernn_batched", 180) == "3_wavernn_batched_180k.wav"
    assert output_name(1, "wavernn_unbatched", 5, input_text="Hello world, again") == \
        "__input_Hello worl_wavernn_unbatched_5k.wav"
    assert output_name(2, "wavernn_batched", 5, standard_name="lj_002") == "lj_002.wav"


def test_synthesize_call_sequence(tmp_path):
    rng = np.random.default_rng(1)
    mels = [rng.uniform(-4, 4, (80, n)).astype(np.float32) for n in (11, 23)]
    tts, voc = _FakeTacotron(mels), _RecordingVocoder()
    attn = []
    synthesize(tts, voc, [0, 1], tmp_path, True, 11000, 550, False, tts_k=7, seed=10,
               save_attention=lambda a, p: attn.append((a, p.name)))
    assert tts.seen == [0, 1]
    assert [c[1].name for c in voc.calls] == ["1_wavernn_batched_7k.wav", "2_wavernn_batched_7k.wav"]
    assert attn == [("attn0", "1_wavernn_batched_7k.wav"), ("attn1", "2_wavernn_batched_7k.wav")]
    for (m, _, batched, target, overlap, mu_law, seed), src, s in zip(voc.calls, mels, (10, 11)):
        assert torch.equal(m, tacotron_mel_to_vocoder(src.copy()))
        assert (batched, target, overlap, mu_law, seed) == (True, 11000, 550, False, s)


def test_saved_mels_checks(tmp_path):
    good = tmp_path / "m.npy"
    np.save(good, np.zeros((80, 5), np.float32))
    bad = tmp_path / "b.npy"
    np.save(bad, np.zeros((64, 5), np.float32))
    src = _SavedMels([good, bad, tmp_path / "x.wav"], 80)
    assert src.generate(0)[1].shape == (80, 5)
    with pytest.raises(ValueError, match="n_mels"):
        src.generate(1)
    with pytest.raises(ValueError, match=".npy"):
        src.generate(2)


@pytest.mark.gpu
def test_synthesize_on_the_dropin(tmp_path):
    """synthesize() through the real drop-in equals vocoding the rescaled mel directly."""
    from wavernn_amd.fatchord_version import WaveRNN
    torch.manual_seed(0)
    voc = WaveRNN(rnn_dims=32, fc_dims=32, bits=9, pad=2, upsample_factors=(5, 5, 11), feat_dims=80,
                  compute_dims=32, res_out_dims=32, res_blocks=2, hop_length=275, sample_rate=22050,
                  mode='MOL').cuda()
    rng = np.random.default_rng(2)
    mels = [rng.uniform(-4, 4, (80, 30)).astype(np.float32)]
    wavs = synthesize(_FakeTacotron(mels), voc, [0], tmp_path, True, 1100, 55, False, seed=5)
    direct = voc.generate(tacotron_mel_to_vocoder(mels[0].copy()), None, True, 1100, 55, False, seed=5,
                          verbose=False)
    assert (tmp_path / "1_wavernn_batched_0k.wav").exists()
    assert np.array_equal(wavs[0], direct)
