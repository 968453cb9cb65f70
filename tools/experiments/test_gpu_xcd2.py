"""The two-rows-per-XCD MoL kernel (csrc/fatchord_xcd2.hip: launch rows k and k + 8 on XCD k, up to
16 rows per launch) through the C-ABI, against the oracle under injected noise (MoL |Δ| <= MOL_TOL).
Row counts: 9..16 (single- and two-row XCDs in one launch), more than one launch (20), time-chunked
launches carrying both rows' state, the fold-batched 5 s utterance's 10 folds over all 12 100 steps
(hparams voc_gen_batched: the reference's default generate() mode), Philox agreement with the
one-row and many-row kernels, row-offset invariance."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
XCD2 = 11   # wrnn_info.last_path


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


def _loop():
    from wavernn_amd.loop import FatchordLoop
    d = syn.DEFAULT_MOL
    return FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)


def _run(B, L, seed, monkeypatch, terms_mb=None):
    from oracle import oracle
    monkeypatch.setenv("WRNN_PATH", "xcd2")
    if terms_mb is not None:
        monkeypatch.setenv("WRNN_TERMS_MB", str(terms_mb))
    d = syn.DEFAULT_MOL
    state = syn.make_fatchord_state(d, seed)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, seed + 1)
    noise = syn.make_noise("MOL", B, L, d.n_classes, seed + 2)
    ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
    loop = _loop()
    loop.set_weights(state)
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == XCD2, loop.info
    err = np.abs(out.cpu().numpy() - ref)
    loop.close()
    return err


@pytest.mark.parametrize("B", [9, 10, 13, 16, 1, 20])
def test_xcd2_vs_oracle(B, monkeypatch):
    err = _run(B, 300, 1100 + B, monkeypatch)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at (row, step) {np.unravel_index(err.argmax(), err.shape)}"


@pytest.mark.parametrize("B", [10, 16])
def test_xcd2_time_chunks_carry_state(B, monkeypatch):
    err = _run(B, 400, 1200 + B, monkeypatch, terms_mb=4)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()}"


def test_xcd2_fold_batched_5s_full_length(monkeypatch):
    """The 10 folds of a 5 s utterance (target 11 000 / overlap 550) over all 12 100 steps."""
    err = _run(10, 12100, 1300, monkeypatch)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


def test_xcd2_is_the_default_for_9_to_16_rows(monkeypatch):
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.DEFAULT_MOL
    state = syn.make_fatchord_state(d, 5)
    loop = _loop()
    loop.set_weights(state)
    for B, path in ((8, 5), (9, XCD2), (16, XCD2), (17, 7)):
        mels, aux = syn.make_conditioning(B, 50, d.feat_dims, d.res_out_dims, 6)
        loop.generate(_cond(mels, aux), seed=1)
        assert loop.info["last_path"] == path, (B, loop.info["last_path"])
    loop.close()


def test_xcd2_agrees_with_other_kernels_under_philox(monkeypatch):
    d = syn.DEFAULT_MOL
    B, L = 12, 500
    state = syn.make_fatchord_state(d, 51)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 52)
    cond = _cond(mels, aux)
    res = {}
    for p in ("xcd2", "xcd", "xcdm"):
        monkeypatch.setenv("WRNN_PATH", p)
        loop = _loop()
        loop.set_weights(state)
        res[p], _ = loop.generate(cond, seed=321, row_offset=3)
        loop.close()
    assert (res["xcd2"] - res["xcd"]).abs().max().item() <= 2 * gf.MOL_TOL
    assert (res["xcd2"] - res["xcdm"]).abs().max().item() <= 2 * gf.MOL_TOL


def test_xcd2_row_offset_invariant(monkeypatch):
    monkeypatch.setenv("WRNN_PATH", "xcd2")
    d = syn.DEFAULT_MOL
    B, L = 14, 300
    state = syn.make_fatchord_state(d, 61)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 62)
    cond = _cond(mels, aux)
    loop = _loop()
    loop.set_weights(state)
    a, _ = loop.generate(cond, seed=9)
    b, _ = loop.generate(cond, seed=9)
    assert torch.equal(a, b)
    r, _ = loop.generate(cond[:, 11:12].contiguous(), seed=9, row_offset=11)
    assert (r[0] - a[11]).abs().max().item() <= gf.MOL_TOL
    loop.close()
