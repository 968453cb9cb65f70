"""Parity of the XCD-resident kernel (fatchord_xcd.hip: one MoL row per XCD, its loop on that
XCD's 32 CUs) through the C-ABI, against the golden fixtures and the oracle.

Tolerance: MoL samples |Δ| <= MOL_TOL (1e-5) per sample under injected noise;
Philox runs of different kernels / launch splits agree within 2·MOL_TOL."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _loop(d):
    from wavernn_amd.loop import FatchordLoop
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
    assert loop.info["xcd_rows"] == 8, loop.info
    return loop


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


def _oracle_case(B, L, seed):
    from oracle import oracle
    d = syn.DEFAULT_MOL
    state = syn.make_fatchord_state(d, seed)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, seed + 1)
    noise = syn.make_noise("MOL", B, L, d.n_classes, seed + 2)
    ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
    return d, state, mels, aux, noise, ref


@pytest.mark.parametrize("name", ["loop_mol_b1", "loop_mol_b4", "loop_mol_1s"])
def test_xcd_vs_reference_fixture(name, monkeypatch):
    """The golden MoL fixtures made by running the reference generate() loop (rnn 512; the 1 s
    fixture runs the full 22 275 steps)."""
    monkeypatch.setenv("WRNN_PATH", "xcd")
    fx = gf.load(name)
    d, state, mels, aux, noise = gf.loop_inputs(fx)
    loop = _loop(d)
    loop.set_weights(state)
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 5
    err = np.abs(out.cpu().numpy() - fx["samples"])
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


@pytest.mark.parametrize("B", [1, 2, 8, 11, 17])
def test_xcd_rows_vs_oracle(B, monkeypatch):
    """One row per XCD, up to 8 per launch: 11 and 17 rows take 2 and 3 launches (rows 8.., 16..
    reuse the XCDs; forced — above 8 rows the many-row kernel is the default); every row
    against the oracle."""
    if B <= 8:
        monkeypatch.delenv("WRNN_PATH", raising=False)    # the default for B <= 8
    else:
        monkeypatch.setenv("WRNN_PATH", "xcd")
    d, state, mels, aux, noise, ref = _oracle_case(B, 300, 110 + B)
    loop = _loop(d)
    loop.set_weights(state)
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 5
    err = np.abs(out.cpu().numpy() - ref)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


def test_xcd_time_chunks_carry_state(monkeypatch):
    """A tiny terms budget splits the utterance into launches that carry h1, the GRU1 terms of
    the next step, W_hh2·h2, h2 and x per workgroup: oracle parity, and Philox output equal to
    the single-launch run within the fp tolerance."""
    monkeypatch.setenv("WRNN_PATH", "xcd")
    d, state, mels, aux, noise, ref = _oracle_case(3, 900, 130)
    loop = _loop(d)
    loop.set_weights(state)
    cond = _cond(mels, aux)
    whole, _ = loop.generate(cond, seed=5)
    monkeypatch.setenv("WRNN_TERMS_MB", "4")      # ~60 steps per launch at 3 rows
    out, _ = loop.generate(cond, noise=torch.from_numpy(noise).to(DEV))
    assert np.abs(out.cpu().numpy() - ref).max() <= gf.MOL_TOL
    chunked, _ = loop.generate(cond, seed=5)
    assert (chunked - whole).abs().max().item() <= 2 * gf.MOL_TOL


@pytest.mark.parametrize("other", ["split", "rows"])
def test_xcd_agrees_with_other_kernels_under_philox(other, monkeypatch):
    """Philox draws are keyed by (seed, global row, step, k) in every kernel: the XCD kernel
    generates the same MoL audio as the role-split and multi-row kernels."""
    d = syn.DEFAULT_MOL
    B = 1 if other == "split" else 3
    L = 1500
    state = syn.make_fatchord_state(d, 141)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 142)
    cond = _cond(mels, aux)
    res = {}
    for p in ("xcd", other):
        monkeypatch.setenv("WRNN_PATH", p)
        loop = _loop(d)
        loop.set_weights(state)
        res[p], _ = loop.generate(cond, seed=91, row_offset=7)
    assert (res["xcd"] - res[other]).abs().max().item() <= 2 * gf.MOL_TOL


def test_xcd_row_offset_sharding_invariance(monkeypatch):
    """Rows [2, 5) generated on their own with row_offset 2 match rows 2..4 of the 5-row run
    (within the fp tolerance: the conditioning-terms GEMM may tile a 3-row batch differently):
    an utterance's audio does not depend on which call / GPU / XCD generated it."""
    monkeypatch.setenv("WRNN_PATH", "xcd")
    d = syn.DEFAULT_MOL
    state = syn.make_fatchord_state(d, 151)
    mels, aux = syn.make_conditioning(5, 500, d.feat_dims, d.res_out_dims, 152)
    cond = _cond(mels, aux)
    loop = _loop(d)
    loop.set_weights(state)
    full, _ = loop.generate(cond, seed=3)
    part, _ = loop.generate(cond[:, 2:].contiguous(), seed=3, row_offset=2)
    assert (full[2:] - part).abs().max().item() <= 2 * gf.MOL_TOL


@pytest.mark.parametrize("B,path", [(1, 5), (8, 5), (9, 7), (49, 7), (200, 7)])
def test_default_path_by_rows(B, path, monkeypatch):
    """Default MoL rnn-512 kernel by row count: one row per XCD (path 5) up to 8 rows, the
    many-row XCD kernel (path 7) above, in launches of up to 128 rows."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.DEFAULT_MOL
    state = syn.make_fatchord_state(d, 161)
    mels, aux = syn.make_conditioning(B, 40, d.feat_dims, d.res_out_dims, 162)
    loop = _loop(d)
    loop.set_weights(state)
    loop.generate(_cond(mels, aux), seed=1)
    assert loop.info["last_path"] == path


def test_xcd_full_headline_length(monkeypatch):
    """The headline workload's full length (BASELINE config 2: 5 s = 110 275 loop steps, one
    row) against the C oracle under injected noise: no drift of the fp32 re-associations over the
    whole utterance (|Δ| <= MOL_TOL at every sample; the oracle takes ~30 s on one core)."""
    monkeypatch.setenv("WRNN_PATH", "xcd")
    L = syn.frames_for_seconds(5.0, syn.DEFAULT_MOL.sample_rate, syn.DEFAULT_MOL.hop_length) * syn.DEFAULT_MOL.hop_length
    assert L == 110275
    d, state, mels, aux, noise, ref = _oracle_case(1, L, 150)
    loop = _loop(d)
    loop.set_weights(state)
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 5
    err = np.abs(out.cpu().numpy() - ref)
    print(f"full-length (110 275 steps) max |Δ| {err.max():.3g}, mean {err.mean():.3g}")
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
