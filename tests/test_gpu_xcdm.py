"""The XCD-resident many-row MoL kernel (csrc/fatchord_xcdm.hip: up to 16 rows per XCD on the
matrix cores, 128 rows per launch) through the C-ABI, against the oracle under injected noise
(MoL |Δ| <= MOL_TOL = 1e-5 per sample, tests/golden/fixtures.py).

Row counts cover one quad per XCD (B <= 32, every workgroup samples every row), the two-level
sampler (B > 32), ragged XCDs (rows not a multiple of 8), the fold-batched 5 s utterance of
BASELINE config 2 (10 folds) over its full 12 100 steps and config 3's 115 folds."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
XCDM = 7   # wrnn_info.last_path


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


def _loop():
    from wavernn_amd.loop import FatchordLoop
    d = syn.DEFAULT_MOL
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
    if loop.info["xcdm_rows"] == 0:
        pytest.skip("many-row XCD kernel unavailable on this device")
    return loop


def _run(B, L, seed, monkeypatch, terms_mb=None):
    from oracle import oracle
    monkeypatch.setenv("WRNN_PATH", "xcdm")
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
    assert loop.info["last_path"] == XCDM, loop.info
    err = np.abs(out.cpu().numpy() - ref)
    loop.close()
    return err


@pytest.mark.parametrize("B", [1, 2, 5, 8, 10, 13, 32, 33, 57, 80, 115, 128])
def test_xcdm_vs_oracle(B, monkeypatch):
    err = _run(B, 240, 700 + B, monkeypatch)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at (row, step) {np.unravel_index(err.argmax(), err.shape)}"


@pytest.mark.parametrize("B", [3, 40])
def test_xcdm_time_chunks_carry_state(B, monkeypatch):
    """A tiny terms budget splits the utterance into several launches that carry h1 / h2 /
    W_hh1·h1 / W_hh2·h2 / x per workgroup (tags continue across launches)."""
    err = _run(B, 400, 800 + B, monkeypatch, terms_mb=4)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()}"


def test_xcdm_more_rows_than_one_launch(monkeypatch):
    """More rows than one launch holds: row blocks of xcdm_rows, each its own launch."""
    loop = _loop()
    n = loop.info["xcdm_rows"]
    loop.close()
    err = _run(n + 7, 120, 900, monkeypatch)
    assert err.max() <= gf.MOL_TOL


def test_xcdm_fold_batched_5s_full_length(monkeypatch):
    """BASELINE config 2 through the reference's default batched path: the 10 folds of a 5 s
    utterance (fold_with_overlap, target 11 000 / overlap 550) over all 12 100 steps."""
    err = _run(10, 12100, 950, monkeypatch)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


@pytest.mark.parametrize("B", [8, 40])
def test_xcdm_agrees_with_other_kernels_under_philox(B, monkeypatch):
    """Philox keyed by (seed, global row, step, k) in every kernel: the many-row kernel, the
    one-row-per-XCD kernel and the HBM rows kernel generate the same audio (fp tolerance)."""
    d = syn.DEFAULT_MOL
    L = 500
    state = syn.make_fatchord_state(d, 31)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 32)
    cond = _cond(mels, aux)
    res = {}
    for p in ("xcdm", "xcd", "rows"):
        monkeypatch.setenv("WRNN_PATH", p)
        loop = _loop()
        loop.set_weights(state)
        res[p], _ = loop.generate(cond, seed=123, row_offset=5)
        loop.close()
    assert (res["xcdm"] - res["xcd"]).abs().max().item() <= 2 * gf.MOL_TOL
    assert (res["xcdm"] - res["rows"]).abs().max().item() <= 2 * gf.MOL_TOL


def test_xcdm_row_offset_invariant(monkeypatch):
    """A row generated alone with its global row id reproduces that row of a batch (Philox)."""
    monkeypatch.setenv("WRNN_PATH", "xcdm")
    d = syn.DEFAULT_MOL
    B, L = 20, 300
    state = syn.make_fatchord_state(d, 41)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 42)
    cond = _cond(mels, aux)
    loop = _loop()
    loop.set_weights(state)
    a, _ = loop.generate(cond, seed=9)
    b, _ = loop.generate(cond, seed=9)
    assert torch.equal(a, b)
    r, _ = loop.generate(cond[:, 13:14].contiguous(), seed=9, row_offset=13)
    assert (r[0] - a[13]).abs().max().item() <= gf.MOL_TOL
    assert float(a.abs().max()) <= 1.0 and torch.isfinite(a).all()
    loop.close()
