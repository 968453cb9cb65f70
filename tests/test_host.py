"""Host-side logic of the drop-in WaveRNN (CPU): state_dict compatibility with the reference
layout, the GPU-side pre-processing (pad → upsample → fold → time-major) against the oracle's
numpy restatement, the float64 post-processing, and the no-CPU-fallback rule."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn
from wavernn_amd.fatchord_version import WaveRNN


def _model(d, seed=0):
    m = WaveRNN(**d.ctor_kwargs())
    state = syn.make_fatchord_state(d, seed)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
    return m, state


def test_state_dict_keys_match_reference_layout():
    for d in (syn.DEFAULT_MOL, syn.DEFAULT_RAW, syn.TINY_RAW):
        m = WaveRNN(**d.ctor_kwargs())
        ours = {k: tuple(v.shape) for k, v in m.state_dict().items()}
        ref = {k: shp for k, (shp, _) in syn.fatchord_state_shapes(d).items()}
        assert ours == ref


@pytest.mark.parametrize("batched", [False, True])
def test_conditioning_matches_oracle(batched):
    d = syn.TINY_MOL
    m, state = _model(d)
    mel = syn.make_mel(d.feat_dims, 24, 3)
    cond, wave_len = m.conditioning(torch.from_numpy(mel)[None], batched, 1500, 200)
    mp = orc.pad_tensor(mel.T[None], d.pad)[0].T
    um, ua = orc.upsample(mp, state, d.upsample_factors, d.res_blocks, d.pad)
    um, ua = um[None], ua[None]
    if batched:
        um, ua = orc.fold_with_overlap(um, 1500, 200), orc.fold_with_overlap(ua, 1500, 200)
    ref = np.concatenate([um, ua], 2).transpose(1, 0, 2)
    assert wave_len == (24 - 1) * d.hop_length
    assert cond.shape == ref.shape
    assert np.abs(cond.numpy() - ref).max() < 1e-5


def test_fold_matches_reference_formula():
    m, _ = _model(syn.TINY_MOL)
    for L, tg, ov in [(1000, 200, 50), (1050, 200, 50), (6600, 1100, 275), (99, 10, 3)]:
        x = torch.arange(L, dtype=torch.float32).reshape(1, L, 1)
        ours = m.fold_with_overlap(x, tg, ov).numpy()
        ref = orc.fold_with_overlap(x.numpy(), tg, ov)
        np.testing.assert_array_equal(ours, ref)


def test_xfade_matches_oracle():
    rng = np.random.default_rng(0)
    y = rng.standard_normal((5, 2000))
    np.testing.assert_array_equal(WaveRNN.xfade_and_unfold(y.copy(), 1500, 250), orc.xfade_and_unfold(y, 250))


def test_generate_refuses_cpu_model():
    m, _ = _model(syn.TINY_MOL)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.generate(torch.rand(1, 80, 24), None, False, 1000, 100, False)


def test_load_roundtrip(tmp_path):
    d = syn.TINY_RAW
    m, _ = _model(d, seed=3)
    p = tmp_path / "w.pyt"
    m.save(p)
    m2 = WaveRNN(**d.ctor_kwargs())
    m2.load(p)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    assert m2.get_step() == 800_000


def test_golden_noise_layout_width():
    fx = gf.load("loop_raw_b1")
    d, _, _, _, noise = gf.loop_inputs(fx)
    m = WaveRNN(**d.ctor_kwargs())
    assert noise.shape[-1] == m.noise_width() == d.n_classes
