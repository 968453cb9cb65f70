"""Parity of the XCD-resident block-sparse kernel (fatchord_xcds.hip: one MoL row of rnn 896 with
4x4 block-sparse GRU weights per XCD, BASELINE config 4) through the C-ABI, against the golden
fixture made by running the reference and against the oracle.

Tolerance: MoL samples |Δ| <= MOL_TOL (1e-5) per sample under injected noise;
Philox runs of different kernels / launch splits agree within 2·MOL_TOL."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn
from wavernn_amd.pruning import prune_state

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _loop(d):
    from wavernn_amd.loop import FatchordLoop
    return FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


def _oracle_case(B, L, seed):
    from oracle import oracle
    d = syn.SPARSE896_MOL
    state = prune_state(syn.make_fatchord_state(d, seed), 0.95)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, seed + 1)
    noise = syn.make_noise("MOL", B, L, d.n_classes, seed + 2)
    ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
    return d, state, mels, aux, noise, ref


def test_xcds_vs_reference_fixture(monkeypatch):
    """The golden rnn-896 95 %-pruned MoL fixture (two rows, made by running the reference)."""
    monkeypatch.delenv("WRNN_PATH", raising=False)        # the default for block-sparse rnn 896
    fx = gf.load("loop_mol_sparse896_b2")
    d, state, mels, aux, noise = gf.loop_inputs(fx)
    loop = _loop(d)
    loop.set_weights(state)
    assert loop.info["xcd_rows"] == 8, loop.info
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 6
    err = np.abs(out.cpu().numpy() - fx["samples"])
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


@pytest.mark.parametrize("B", [1, 3, 9])
def test_xcds_rows_vs_oracle(B, monkeypatch):
    """One row per XCD, 8 per launch (9 rows: two launches); every row against the oracle."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d, state, mels, aux, noise, ref = _oracle_case(B, 300, 610 + B)
    loop = _loop(d)
    loop.set_weights(state)
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 6
    err = np.abs(out.cpu().numpy() - ref)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


def test_xcds_time_chunks(monkeypatch):
    """Time-chunked launches (the recurrent state carried per workgroup) match the oracle and a
    single launch."""
    d, state, mels, aux, noise, ref = _oracle_case(2, 700, 640)
    loop = _loop(d)
    loop.set_weights(state)
    cond = _cond(mels, aux)
    whole, _ = loop.generate(cond, seed=3)
    monkeypatch.setenv("WRNN_TERMS_MB", "4")      # ~150 steps per launch at 2 rows
    out, _ = loop.generate(cond, noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 6
    assert np.abs(out.cpu().numpy() - ref).max() <= gf.MOL_TOL
    chunked, _ = loop.generate(cond, seed=3)
    assert (chunked - whole).abs().max().item() <= 2 * gf.MOL_TOL


def test_xcds_agrees_with_rows_kernel_under_philox(monkeypatch):
    """Same Philox keying as the multi-row kernel (sparse blocks there too): the same audio
    within the fp tolerance, rows offset by a global row id."""
    d = syn.SPARSE896_MOL
    B, L = 3, 1500
    state = prune_state(syn.make_fatchord_state(d, 650), 0.95)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 651)
    cond = _cond(mels, aux)
    res = {}
    for p, path in (("xcd", 6), ("rows", 2)):
        monkeypatch.setenv("WRNN_PATH", p)
        loop = _loop(d)
        loop.set_weights(state)
        res[p], _ = loop.generate(cond, seed=17, row_offset=5)
        assert loop.info["last_path"] == path
    assert (res["xcd"] - res["rows"]).abs().max().item() <= 2 * gf.MOL_TOL


def test_xcds_one_second_vs_oracle(monkeypatch):
    """A full 1 s utterance (22 275 loop steps, one row) of config 4's sparse rnn-896 model against
    the C oracle under injected noise: no drift over the utterance."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    L = syn.frames_for_seconds(1.0) * 275
    assert L == 22275
    d, state, mels, aux, noise, ref = _oracle_case(1, L, 640)
    loop = _loop(d)
    loop.set_weights(state)
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 6
    err = np.abs(out.cpu().numpy() - ref)
    print(f"sparse 1 s (22 275 steps) max |Δ| {err.max():.3g}, mean {err.mean():.3g}")
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


def test_xcds_five_seconds_vs_oracle_fixture(monkeypatch):
    """Config 4 at its own length: a whole 5 s utterance (110 275 steps) of the 95 %-pruned
    rnn-896 model through the sparse XCD kernel against the C oracle's full-length output
    (tests/golden/long_sparse896_5s.npz, make_long_fixtures.py; the oracle is pinned to the
    reference by the reference fixtures), under the same injected noise: no drift."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    fx = gf.load("long_sparse896_5s")
    d, state, mels, aux, noise = gf.loop_inputs(fx)
    assert int(fx["L"]) == 110275
    loop = _loop(d)
    loop.set_weights(state)
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 6
    err = np.abs(out.cpu().numpy()[fx["full_rows"]] - fx["out_full"])
    print(f"sparse 5 s (110 275 steps) vs oracle: max |Δ| {err.max():.3g}, mean {err.mean():.3g}")
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
    loop.close()
