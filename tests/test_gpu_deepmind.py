"""deepmind_version (config 5 model) on the MI355X dual-softmax kernel: coarse/fine labels and
the combined 16-bit output bit-exact vs the reference fixtures and the oracle."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("name", gf.DM_CASES)
def test_dm_loop_vs_reference_fixture(name):
    from wavernn_amd.loop import DeepmindLoop
    fx = gf.load(name)
    d, state, noise = gf.dm_inputs(fx)
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(state)
    L = int(fx["L"])
    out, comb = loop.generate(1, L, noise=torch.from_numpy(noise).to(DEV))
    comb = comb.cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(comb, fx["output"].astype(np.int64))
    np.testing.assert_array_equal(out.cpu().numpy(), comb.astype(np.float32))


@pytest.mark.parametrize("name", gf.DM_CASES)
def test_dm_generate_dropin_vs_reference(name):
    from wavernn_amd.deepmind_version import WaveRNN
    fx = gf.load(name)
    d, state, noise = gf.dm_inputs(fx)
    m = WaveRNN(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()}, strict=True)
    output, coarse, fine = m.generate(int(fx["L"]), noise=noise)
    np.testing.assert_array_equal(coarse, fx["coarse"][0].astype(np.int64))
    np.testing.assert_array_equal(fine, fx["fine"][0].astype(np.int64))
    np.testing.assert_array_equal(output, fx["output"][0].astype(np.int64))


@pytest.mark.parametrize("d,B,L", [(syn.DEFAULT_DM, 5, 400), (syn.TINY_DM, 40, 200)])
def test_dm_many_rows_vs_oracle(d, B, L):
    """Independent rows (config 5's utterance batch) in one launch; tiny dims put several
    sampled rows on each of its 32 workgroups."""
    from oracle import oracle
    from wavernn_amd.loop import DeepmindLoop
    state = syn.make_deepmind_state(d, 11)
    noise = syn.make_dm_noise(B, L, d.quantisation, 12)
    _, _, ref = oracle.deepmind_loop(state, B, L, noise)
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(state)
    _, comb = loop.generate(B, L, noise=torch.from_numpy(noise).to(DEV))
    got = comb.cpu().numpy().astype(np.int64)
    eq = got == ref
    assert eq.all(), f"{eq.mean():.6f} equal, first mismatch {np.argwhere(~eq)[0].tolist()}"


def test_dm_philox_row_keyed():
    """Philox draws keyed by (seed, global row, step, k): row 2 alone reproduces row 2 of a batch."""
    from wavernn_amd.loop import DeepmindLoop
    d = syn.DEFAULT_DM
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(syn.make_deepmind_state(d, 13))
    _, a = loop.generate(3, 300, seed=99)
    _, b = loop.generate(3, 300, seed=99)
    _, r2 = loop.generate(1, 300, seed=99, row_offset=2)
    assert torch.equal(a, b)
    assert torch.equal(r2[0], a[2])
    u = a.cpu().numpy() + 2 ** 15
    assert (u >= 0).all() and (u < 2 ** 16).all() and len(np.unique(u // 256)) > 100


def test_dm_row_groups_agree(monkeypatch):
    """One group of G workgroups vs two groups of G/2 (twice the units each): the coarse/fine
    labels are bit-exact across partitions (Philox keyed by global row).  Multi-row kernel forced
    (hidden 896 defaults to the XCD-resident kernel)."""
    from wavernn_amd.loop import DeepmindLoop
    monkeypatch.setenv("WRNN_PATH", "rows")
    d = syn.DEFAULT_DM
    res = {}
    for g in ("1", "2"):
        monkeypatch.setenv("WRNN_ROW_GROUPS", g)
        loop = DeepmindLoop(d.hidden_size, d.quantisation)
        loop.set_weights(syn.make_deepmind_state(d, 17))
        res[g] = loop.generate(9, 300, seed=5)[1]
        loop.close()
    assert torch.equal(res["1"], res["2"])


@pytest.mark.gpu
@pytest.mark.parametrize("B", [3, 20, 40])
def test_dm_granule_and_bulk_handoffs(B, monkeypatch):
    """Granule hand-offs (small row groups) and bulk flag + DMA hand-offs, both forced: the
    combined labels are bit-exact between the two (Philox keyed by global row).  Multi-row
    kernel forced."""
    from wavernn_amd.loop import DeepmindLoop
    monkeypatch.setenv("WRNN_PATH", "rows")
    d = syn.DEFAULT_DM
    res = {}
    for g in ("0", "1"):
        monkeypatch.setenv("WRNN_ROWS_GRANULES", g)
        loop = DeepmindLoop(d.hidden_size, d.quantisation)
        loop.set_weights(syn.make_deepmind_state(d, 23))
        res[g] = loop.generate(B, 300, seed=7)[1]
        loop.close()
    assert torch.equal(res["0"], res["1"])


def test_dm_full_second_bit_exact():
    """Config 5's full utterance length (1 s at 16 kHz = 16 000 steps), 2 rows, H = 896: every
    coarse/fine label and combined sample bit-exact vs the oracle under injected noise."""
    from oracle import oracle
    from wavernn_amd.loop import DeepmindLoop
    d, B, L = syn.DEFAULT_DM, 2, 16000
    state = syn.make_deepmind_state(d, 21)
    noise = syn.make_dm_noise(B, L, d.quantisation, 22)
    _, _, ref = oracle.deepmind_loop(state, B, L, noise)
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(state)
    _, comb = loop.generate(B, L, noise=torch.from_numpy(noise).to(DEV))
    got = comb.cpu().numpy().astype(np.int64)
    eq = got == ref
    assert eq.all(), f"{eq.mean():.6f} equal, first mismatch {np.argwhere(~eq)[0].tolist()}"
    loop.close()
