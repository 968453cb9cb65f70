"""The XCD-resident deepmind kernel (deepmind_xcd.hip, path 8: hidden 896, quantisation 256, up
to 4 rows per XCD and 32 per launch, weights as fp32 MFMA operands) against the C oracle
(coarse/fine labels and the combined 16-bit output bit-exact), against the multi-row kernel
under Philox, across launches of 32 rows and across time chunks."""
import numpy as np
import pytest
import torch

from oracle import oracle
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _loop(d):
    from wavernn_amd.loop import DeepmindLoop
    return DeepmindLoop(d.hidden_size, d.quantisation)


def _check(comb, ref):
    comb = comb.cpu().numpy().astype(np.int64)
    eq = comb == ref
    assert eq.all(), f"{eq.mean():.6f} equal, first mismatch {np.argwhere(~eq)[0].tolist()}"


@pytest.mark.parametrize("B,L", [(1, 300), (4, 200), (8, 200), (9, 200), (17, 150), (32, 150), (40, 100)])
def test_dx_vs_oracle(B, L, monkeypatch):
    """Injected draws; 40 rows take two launches (32 + 8)."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.DEFAULT_DM
    state = syn.make_deepmind_state(d, 31 + B)
    noise = syn.make_dm_noise(B, L, d.quantisation, 32 + B)
    _, _, ref = oracle.deepmind_loop(state, B, L, noise)
    loop = _loop(d)
    loop.set_weights(state)
    out, comb = loop.generate(B, L, noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 8
    _check(comb, ref)
    np.testing.assert_array_equal(out.cpu().numpy(), comb.cpu().numpy().astype(np.float32))
    loop.close()


def test_dx_matches_rows_kernel_under_philox(monkeypatch):
    """Philox draws are keyed by (seed, global row, step, k) in both deepmind kernels: the same
    labels from the XCD-resident and the multi-row kernel."""
    d = syn.DEFAULT_DM
    state = syn.make_deepmind_state(d, 41)
    res = {}
    for p in ("", "rows"):
        monkeypatch.setenv("WRNN_PATH", p)
        loop = _loop(d)
        loop.set_weights(state)
        res[p] = loop.generate(11, 500, seed=8, row_offset=3)[1]
        assert loop.info["last_path"] == (8 if p == "" else 3)
        loop.close()
    assert torch.equal(res[""], res["rows"])


def test_dx_time_chunks_carry_state(monkeypatch):
    """A tiny draws budget splits the utterance into launches that carry h, the R·h partials and
    the previous labels per workgroup: labels identical to the single-launch run."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.DEFAULT_DM
    loop = _loop(d)
    loop.set_weights(syn.make_deepmind_state(d, 43))
    whole = loop.generate(6, 700, seed=4)[1]
    monkeypatch.setenv("WRNN_DM_NOISE_MB", "1")      # ~85 steps per launch at 6 rows
    chunked = loop.generate(6, 700, seed=4)[1]
    assert torch.equal(whole, chunked)
    loop.close()


def test_dx_row_offset_invariance(monkeypatch):
    """Row 2 alone (row_offset 2) reproduces row 2 of a 5-row batch: an utterance's audio does not
    depend on which launch, XCD or GPU generated it."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.DEFAULT_DM
    loop = _loop(d)
    loop.set_weights(syn.make_deepmind_state(d, 47))
    full = loop.generate(5, 400, seed=12)[1]
    part = loop.generate(1, 400, seed=12, row_offset=2)[1]
    assert torch.equal(full[2], part[0])
    loop.close()
