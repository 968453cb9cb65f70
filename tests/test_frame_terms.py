"""The frame-rate form of the UpsampleNetwork's mel path (wrnn_frame_weights, csrc/capi.cpp;
csrc/frame_terms.hip): mel_up(f·hop + φ) = Σ_k coef[φ][k]·mel[f + k + jlo] must reproduce the
stage-wise Stretch2d/Conv2d cascade (fatchord_version.py:64-89, restated by oracle.upsample) —
host-only, no GPU.  The GPU side (the terms formed from these weights inside the loop entry) is
tests/test_gpu_frame_terms.py."""
import numpy as np
import pytest

from oracle import oracle
from wavernn_amd import _native as nat
from wavernn_amd import condition
from wavernn_amd import synthetic as syn


def _mel_up_frames(mel, jlo, coef, hop):
    """Σ_k coef[φ][k]·mel[:, f + k + jlo] in float64, [L][feat]."""
    feat, T = mel.shape
    nJ = coef.shape[1]
    p = np.arange(T * hop)
    f, ph = p // hop, p % hop
    out = np.zeros((T * hop, feat))
    for k in range(nJ):
        fr = f + k + jlo
        ok = (fr >= 0) & (fr < T)
        out[ok] += coef[ph[ok], k][:, None].astype(np.float64) * mel[:, fr[ok]].T.astype(np.float64)
    return out


def _oracle_mel_up(mel, taps, scales, pad):
    state = {f"upsample.up_layers.{2 * i + 1}.weight": np.asarray(t, np.float32).reshape(1, 1, 1, -1)
             for i, t in enumerate(taps)}
    mp = oracle.pad_tensor(mel.T[None], pad)[0].T            # [feat][T + 2pad]
    total = int(np.prod(scales))
    m = mp.astype(np.float64)                                 # the cascade of oracle.upsample (mel part)
    for i, s in enumerate(scales):
        m = np.repeat(m, s, axis=1)
        kern = state[f"upsample.up_layers.{2 * i + 1}.weight"].reshape(-1).astype(np.float64)
        mpad = np.pad(m, ((0, 0), (s, s)))
        m = sum(kern[j] * mpad[:, j:j + m.shape[1]] for j in range(2 * s + 1))
    return m[:, pad * total:-pad * total].T


@pytest.mark.parametrize("case", ["box", "random", "small"])
def test_frame_weights_reproduce_the_cascade(case):
    rng = np.random.default_rng(7)
    if case == "small":
        scales, pad = (2, 3), 2
    else:
        scales, pad = (5, 5, 11), 2
    if case == "box":
        st = syn.make_fatchord_state(syn.DEFAULT_MOL, 0)
        taps = [st[f"upsample.up_layers.{2 * i + 1}.weight"].reshape(-1) for i in range(3)]
    else:
        taps = [(rng.standard_normal(2 * s + 1) * 0.3 + 1.0 / (2 * s + 1)).astype(np.float32) for s in scales]
    spec = condition.UpsampleSpec(80, 128, pad, scales, taps)
    jlo, nJ, coef = condition.frame_weights(spec)
    hop = int(np.prod(scales))
    assert coef.shape == (hop, nJ) and nJ <= 8
    mel = rng.standard_normal((80, 9)).astype(np.float32)
    want = _oracle_mel_up(mel, taps, scales, pad)
    got = _mel_up_frames(mel, jlo, coef, hop)
    # coef rounded to fp32 (relative 6e-8 each); the stage-wise cascade in float64
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-6 * np.abs(want).max())


def test_box_weights_shape_for_the_reference_hparams():
    """(5, 5, 11), pad 2 (hparams voc_upsample_factors / voc_pad): the response reaches 341
    samples before and 615 after a frame's first sample → frames f − 2 … f + 2."""
    st = syn.make_fatchord_state(syn.DEFAULT_MOL, 0)
    taps = [st[f"upsample.up_layers.{2 * i + 1}.weight"].reshape(-1) for i in range(3)]
    jlo, nJ, coef = condition.frame_weights(condition.UpsampleSpec(80, 128, 2, (5, 5, 11), taps))
    assert (jlo, nJ) == (-2, 5)
    # a constant mel is scaled by the product of the stages' tap sums (1 for exact box taps)
    gain = np.prod([t.astype(np.float64).sum() for t in taps])
    np.testing.assert_allclose(coef.astype(np.float64).sum(1), gain, rtol=1e-6)


def test_short_pad_has_no_exact_frame_form():
    """pad 1 frame (275 samples) < the cascade's 341-sample reach: the stage-wise zero padding
    differs from the frame-level one, so the loop entry keeps the per-sample conditioning."""
    taps = [np.full(2 * s + 1, 1.0 / (2 * s + 1), np.float32) for s in (5, 5, 11)]
    with pytest.raises(nat.WrnnError):
        condition.frame_weights(condition.UpsampleSpec(80, 128, 1, (5, 5, 11), taps))
