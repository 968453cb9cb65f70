"""The loop entry from frames (wrnn_generate_frames: conditioning terms formed at frame rate,
csrc/frame_terms.hip) against the per-sample entry (wrnn_upsample_pack → wrnn_generate) on the
MI355X, path by path.  The two differ only in how the terms W·[mel_up | aux | 1] are rounded
(W·mel per frame then the cascade's frame weights, vs the upsampled mel then W), so MoL samples
agree within the tolerance used between launches of different shapes (2·MOL_TOL) and RAW labels
exactly; WRNN_NO_FRAME_TERMS=1 makes the frames entry take the per-sample route, bit for bit.
Oracle parity of the drop-in generate() (which now takes this entry) is tests/test_gpu_parity.py
and tests/test_gpu_baseline_shapes.py.  Reference: fatchord_version.py:169-241."""
import os

import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf

from wavernn_amd import condition
from wavernn_amd import synthetic as syn
from wavernn_amd.pruning import prune_state

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(d, seed, prune=0.0):
    from wavernn_amd.fatchord_version import WaveRNN
    st = syn.make_fatchord_state(d, seed)
    if prune:
        st = prune_state(st, prune)
    m = WaveRNN(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in st.items()})
    return m


def _both(m, n_utt, frames, target, overlap, seed, want_labels=False):
    mel = torch.cat([torch.from_numpy(syn.make_mel(m.feat_dims, frames, 90 + i))[None] for i in range(n_utt)], 0)
    mel_f, aux, _ = m.frames(mel.to(DEV))
    spec = m._upsample_spec()
    loop = m.loop_handle()
    got, glab = loop.generate_frames(spec, mel_f, aux, target, overlap, seed=seed, want_labels=want_labels)
    path_f = loop.info["last_path"]
    cond = condition.upsample_pack(spec, mel_f, aux, target, overlap)
    ref, rlab = loop.generate(cond, seed=seed, want_labels=want_labels)
    assert loop.info["last_path"] == path_f
    assert got.shape == ref.shape
    return got.cpu().numpy(), ref.cpu().numpy(), glab, rlab, path_f


def _close(a, b, what):
    err = float(np.abs(a - b).max())
    print(f"{what}: max |Δ| {err:.3g}")
    assert err <= 2 * gf.MOL_TOL, (what, err)


def test_frames_xcd_unbatched_and_eight_utterances():
    m = _model(syn.DEFAULT_MOL, 3)
    for n_utt in (1, 8):
        got, ref, _, _, path = _both(m, n_utt, 24, 0, 0, seed=11)
        assert path == 5
        _close(got, ref, f"xcd, {n_utt} utterances")


def test_frames_xcd_fold_batched_tail():
    """Folds whose window runs past the utterance: the tail steps take W·[0 | 0 | 1]."""
    m = _model(syn.DEFAULT_MOL, 4)
    got, ref, _, _, path = _both(m, 1, 50, 4000, 200, seed=12)   # 13 750 samples → 4 folds (last one padded)
    assert path == 5 and got.shape[0] == 4
    _close(got, ref, "xcd folds")


def test_frames_xcds_sparse896():
    m = _model(syn.SPARSE896_MOL, 0, prune=0.95)
    got, ref, _, _, path = _both(m, 2, 12, 0, 0, seed=13)
    assert path == 6
    _close(got, ref, "xcds")


def test_frames_xcdm_fold_batched():
    m = _model(syn.DEFAULT_MOL, 5)
    got, ref, _, _, path = _both(m, 1, 60, 1200, 100, seed=14)   # 16 500 samples → 12 folds
    assert path == 7 and got.shape[0] >= 9
    _close(got, ref, "xcdm folds")


def test_frames_xcdm_raw_labels_exact():
    m = _model(syn.DEFAULT_RAW, 6)
    got, ref, glab, rlab, path = _both(m, 1, 24, 0, 0, seed=15, want_labels=True)
    assert path == 7
    mism = int((glab != rlab).sum().item())
    assert mism == 0, f"{mism} RAW labels differ between the frame-rate and per-sample terms"
    np.testing.assert_array_equal(got, ref)


def test_frames_single_fold_longer_than_the_utterance():
    """target past the utterance: one fold (fold_with_overlap's remainder branch), most of its
    window the zero tail."""
    m = _model(syn.DEFAULT_MOL, 8)
    got, ref, _, _, path = _both(m, 1, 30, 20000, 550, seed=17)   # 8 250 samples, window 21 100
    assert got.shape == (1, 21100) and path == 5
    _close(got, ref, "single fold")


def test_frames_entry_on_a_non_xcd_path_takes_the_records():
    """Dims no XCD-resident kernel runs (rnn 64): wrnn_generate_frames builds the per-sample
    records itself (wrnn_upsample_pack into a handle workspace) — bit-identical to the two calls."""
    m = _model(syn.TINY_MOL, 2)
    got, ref, _, _, path = _both(m, 2, 14, 0, 0, seed=18)
    assert path not in (5, 6, 7)
    np.testing.assert_array_equal(got, ref)


def test_frames_env_fallback_is_the_per_sample_route(monkeypatch):
    monkeypatch.setenv("WRNN_NO_FRAME_TERMS", "1")
    m = _model(syn.DEFAULT_MOL, 3)
    got, ref, _, _, path = _both(m, 2, 16, 0, 0, seed=16)
    assert path == 5
    np.testing.assert_array_equal(got, ref)


def test_frames_rejects_mismatched_inputs():
    from wavernn_amd import _native as nat
    m = _model(syn.DEFAULT_MOL, 3)
    mel_f, aux, _ = m.frames(torch.from_numpy(syn.make_mel(80, 10, 1))[None].to(DEV))
    loop = m.loop_handle()
    with pytest.raises(ValueError):
        loop.generate_frames(m._upsample_spec(), mel_f, aux[:, :64].contiguous())
    bad = condition.UpsampleSpec(80, 64, 2, (5, 5, 11), [np.ones(2 * s + 1, np.float32) for s in (5, 5, 11)])
    with pytest.raises(nat.WrnnError):
        nat.check(loop._h, nat.lib().wrnn_generate_frames(loop._h, __import__("ctypes").byref(bad.cfg),
                                                          mel_f.data_ptr(), aux.data_ptr(), 1, 10, 0, 0, None, 0, 0,
                                                          torch.empty(1, 2750, device=DEV).data_ptr(), None, None))
