"""Edge cases of every loop kernel through the C-ABI, against the oracle under injected noise:
the shortest utterances (1 and 2 loop steps — the reference's generate() loop runs
`for i in range(seq_len)` with seq_len = mel frames × hop, fatchord_version.py:199, so any
length ≥ 1 reaches the loop), a launch per step (a terms budget so small that every time chunk is
one step: the carried state h1 / h2 / recurrent sums / x / tags cross a launch boundary at every
step), and the argument errors the C-ABI reports instead of launching (B = 0, L = 0, wrong shapes).

MoL |Δ| <= MOL_TOL (1e-5); RAW labels and deepmind labels bit-exact."""
import numpy as np
import pytest
import torch

from oracle import oracle
from tests.golden import fixtures as gf
from wavernn_amd import _native as nat
from wavernn_amd import synthetic as syn
from wavernn_amd.pruning import prune_state

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
# WRNN_PATH → wrnn_info.last_path (capi.cpp, wrnn_generate)
MOL_PATHS = {"latency": 1, "rows": 2, "split": 4, "xcd": 5, "xcdm": 7}
RAW_PATHS = {"latency": 1, "rows": 2, "xcdm": 7}
TINY_BUDGET_MB = "0.0001"   # every time chunk one step


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


def _fatchord(d, state, path, B, L, seed, monkeypatch, budget=None):
    from wavernn_amd.loop import FatchordLoop
    monkeypatch.setenv("WRNN_PATH", path)
    if budget is not None:
        monkeypatch.setenv("WRNN_TERMS_MB", budget)
    else:
        monkeypatch.delenv("WRNN_TERMS_MB", raising=False)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, seed + 1)
    noise = syn.make_noise(d.mode, B, L, d.n_classes, seed + 2)
    ref, ref_lab = oracle.fatchord_loop(state, d.mode, mels, aux, noise)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
    loop.set_weights(state)
    out, lab = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=d.mode == "RAW")
    info = loop.info
    loop.close()
    return info, out.cpu().numpy(), (lab.cpu().numpy() if lab is not None else None), ref, ref_lab


def _expect_path(info, path, ids):
    want = ids[path]
    if path == "rows" and info["last_path"] == 9:   # streamed-weights rows instantiation
        want = 9
    assert info["last_path"] == want, (path, info["last_path"])


@pytest.mark.parametrize("path", list(MOL_PATHS))
@pytest.mark.parametrize("L", [1, 2])
def test_mol_shortest_utterances(path, L, monkeypatch):
    d = syn.DEFAULT_MOL
    state = syn.make_fatchord_state(d, 1100 + L)
    for B in ((1,) if path == "split" else (1, 3)):
        info, out, _, ref, _ = _fatchord(d, state, path, B, L, 1200 + B, monkeypatch)
        _expect_path(info, path, MOL_PATHS)
        assert out.shape == (B, L)
        assert np.abs(out - ref).max() <= gf.MOL_TOL, (path, B, L, np.abs(out - ref).max())


@pytest.mark.parametrize("path", list(RAW_PATHS))
@pytest.mark.parametrize("L", [1, 2])
def test_raw_shortest_utterances(path, L, monkeypatch):
    d = syn.DEFAULT_RAW
    state = syn.make_fatchord_state(d, 1300 + L)
    for B in (1, 3):
        info, out, lab, ref, ref_lab = _fatchord(d, state, path, B, L, 1400 + B, monkeypatch)
        _expect_path(info, path, RAW_PATHS)
        np.testing.assert_array_equal(lab, ref_lab)
        np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("path", list(MOL_PATHS))
def test_mol_one_step_per_launch(path, monkeypatch):
    """Every time chunk one step: state and tags carried across 7 launches."""
    d = syn.DEFAULT_MOL
    state = syn.make_fatchord_state(d, 1500)
    B = 1 if path == "split" else 5
    info, out, _, ref, _ = _fatchord(d, state, path, B, 7, 1510, monkeypatch, budget=TINY_BUDGET_MB)
    _expect_path(info, path, MOL_PATHS)
    assert np.abs(out - ref).max() <= gf.MOL_TOL, (path, np.abs(out - ref).max())


@pytest.mark.parametrize("path", list(RAW_PATHS))
def test_raw_one_step_per_launch(path, monkeypatch):
    d = syn.DEFAULT_RAW
    state = syn.make_fatchord_state(d, 1600)
    info, _, lab, _, ref_lab = _fatchord(d, state, path, 4, 6, 1610, monkeypatch, budget=TINY_BUDGET_MB)
    _expect_path(info, path, RAW_PATHS)
    np.testing.assert_array_equal(lab, ref_lab)


@pytest.mark.parametrize("L", [1, 2, 5])
def test_sparse896_xcds_short(L, monkeypatch):
    d = syn.SPARSE896_MOL
    state = prune_state(syn.make_fatchord_state(d, 1700 + L), 0.95)
    info, out, _, ref, _ = _fatchord(d, state, "", 2, L, 1710 + L, monkeypatch,
                                     budget=TINY_BUDGET_MB if L == 5 else None)
    if info["last_path"] != 6:
        pytest.skip(f"sparse XCD kernel not selected (path {info['last_path']})")
    assert np.abs(out - ref).max() <= gf.MOL_TOL


@pytest.mark.parametrize("path,pid", [("", 8), ("rows", 3)])
@pytest.mark.parametrize("B,L", [(1, 1), (3, 2), (5, 7)])
def test_deepmind_short(path, pid, B, L, monkeypatch):
    from wavernn_amd.loop import DeepmindLoop
    monkeypatch.setenv("WRNN_PATH", path)
    if L == 7:
        monkeypatch.setenv("WRNN_TERMS_MB", TINY_BUDGET_MB)
    d = syn.DEFAULT_DM
    state = syn.make_deepmind_state(d, 1800 + B)
    noise = syn.make_dm_noise(B, L, d.quantisation, 1810 + B)
    _, _, ref = oracle.deepmind_loop(state, B, L, noise)
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(state)
    _, comb = loop.generate(B, L, noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] in (pid, 10 if pid == 3 else pid)
    loop.close()
    np.testing.assert_array_equal(comb.cpu().numpy().astype(np.int64), ref)


def test_argument_errors_do_not_launch():
    """B = 0 / L = 0 and mismatched shapes are rejected before any launch, and the handle stays
    usable afterwards."""
    from wavernn_amd.loop import DeepmindLoop, FatchordLoop
    d = syn.DEFAULT_MOL
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
    loop.set_weights(syn.make_fatchord_state(d, 1900))
    C = loop.cond_dims
    with pytest.raises(nat.WrnnError):
        loop.generate(torch.zeros(0, 1, C, device=DEV))
    with pytest.raises(nat.WrnnError):
        loop.generate(torch.zeros(4, 0, C, device=DEV))
    with pytest.raises(ValueError):
        loop.generate(torch.zeros(4, 1, C + 1, device=DEV))
    with pytest.raises(ValueError):
        loop.generate(torch.zeros(4, 1, C, device=DEV), noise=torch.zeros(4, 1, 3, device=DEV))
    out, _ = loop.generate(torch.zeros(4, 1, C, device=DEV), seed=1)   # still usable
    assert out.shape == (1, 4) and torch.isfinite(out).all()
    loop.close()
    dm = DeepmindLoop(syn.DEFAULT_DM.hidden_size, syn.DEFAULT_DM.quantisation)
    dm.set_weights(syn.make_deepmind_state(syn.DEFAULT_DM, 1901))
    with pytest.raises(nat.WrnnError):
        dm.generate(0, 10)
    with pytest.raises(nat.WrnnError):
        dm.generate(2, 0)
    _, comb = dm.generate(2, 3, seed=1)
    assert comb.shape == (2, 3)
    dm.close()
