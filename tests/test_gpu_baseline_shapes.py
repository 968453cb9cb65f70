"""Parity at BASELINE.json's own multi-row shapes, through whatever kernel the default path picks.

* config 3 (MoL rnn 512, one 60 s utterance fold-batched = 115 rows of 12 100 steps): all 115
  rows in one generate() call, 300 steps, MoL |Δ| <= MOL_TOL vs the oracle; the RAW 9-bit model
  at the same row count, labels bit-exact; and the whole 12 100 steps of all 115 rows against the
  C oracle's full-length fixture (tests/golden/long_mol_fold115.npz: rows 0/7/64/114 at every
  step, every row at every 50th).
* config 5 (deepmind 896/256, 32 utterances per GPU): 32 rows × 1 000 steps, every coarse/fine
  label and combined sample bit-exact vs the oracle (deepmind_version.py:98-156).
Injected noise in the reference draw order; tolerances as tests/golden/fixtures.py."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


@pytest.mark.parametrize("mode", ["MOL", "RAW"])
def test_config3_115_rows_vs_oracle(mode):
    from oracle import oracle
    from wavernn_amd.loop import FatchordLoop
    d = syn.DEFAULT_MOL if mode == "MOL" else syn.DEFAULT_RAW
    B, L = 115, 300
    state = syn.make_fatchord_state(d, 301)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 302)
    noise = syn.make_noise(mode, B, L, d.n_classes, 303)
    ref, ref_lab = oracle.fatchord_loop(state, mode, mels, aux, noise)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
    loop.set_weights(state)
    out, lab = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=(mode == "RAW"))
    if mode == "RAW":
        got = lab.cpu().numpy()
        eq = got == ref_lab
        assert eq.all(), f"{eq.mean():.6f} equal, first mismatch (row, step) {np.argwhere(~eq)[0].tolist()}"
    else:
        err = np.abs(out.cpu().numpy() - ref)
        assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
    loop.close()


def test_config5_32_rows_bit_exact():
    from oracle import oracle
    from wavernn_amd.loop import DeepmindLoop
    d, B, L = syn.DEFAULT_DM, 32, 1000
    state = syn.make_deepmind_state(d, 501)
    noise = syn.make_dm_noise(B, L, d.quantisation, 502)
    _, _, ref = oracle.deepmind_loop(state, B, L, noise)
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(state)
    _, comb = loop.generate(B, L, noise=torch.from_numpy(noise).to(DEV))
    got = comb.cpu().numpy().astype(np.int64)
    eq = got == ref
    assert eq.all(), f"{eq.mean():.6f} equal, first mismatch {np.argwhere(~eq)[0].tolist()}"
    loop.close()


def test_config3_115_rows_full_length_vs_oracle_fixture():
    """No drift at 115 rows over a whole fold (12 100 steps): the many-row kernel against the C
    oracle's output (make_long_fixtures.py), same injected noise."""
    from wavernn_amd.loop import FatchordLoop
    fx = gf.load("long_mol_fold115")
    d, state, mels, aux, noise = gf.loop_inputs(fx)
    assert (int(fx["B"]), int(fx["L"])) == (115, 12100)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
    loop.set_weights(state)
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 7
    got = out.cpu().numpy()
    sub = int(fx["sub"])
    for name, a, b in (("full rows", got[fx["full_rows"]], fx["out_full"]), ("every row", got[:, ::sub], fx["out_sub"])):
        err = np.abs(a - b)
        print(f"config 3 {name}: max |Δ| {err.max():.3g}, mean {err.mean():.3g}")
        assert err.max() <= gf.MOL_TOL, f"{name}: max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
    loop.close()
