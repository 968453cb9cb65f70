"""Block-sparse pruning (wavernn_amd/pruning.py), BASELINE config 4 / SURVEY.md §8 a16."""
import numpy as np

from wavernn_amd import pruning, synthetic as syn


def _elementwise_reference_rule(W, z, splits=3):
    """notebooks/Pruning - Scratchpad.ipynb PruneMask.mask_from_matrix, restated in numpy:
    per gate split, k = int(numel·z), threshold = sorted(|W|)[k], keep |W| >= threshold."""
    out = []
    for Wg in np.split(W, splits):
        a = np.abs(Wg)
        thr = np.sort(a.reshape(-1))[int(a.size * z)]
        out.append((a >= thr).astype(np.float32))
    return np.concatenate(out)


def test_block_size_one_is_the_notebooks_elementwise_rule():
    W = np.random.default_rng(0).standard_normal((3 * 16, 24)).astype(np.float32)
    for z in (0.0, 0.5, 0.9375):
        np.testing.assert_array_equal(pruning.block_mask(W, z, block=1), _elementwise_reference_rule(W, z))


def test_block_mask_zeroes_whole_blocks_per_gate():
    W = np.random.default_rng(1).standard_normal((3 * 64, 96)).astype(np.float32)
    M = pruning.block_mask(W, 0.95)
    blocks = M.reshape(3 * 16, 4, 24, 4)
    assert np.all((blocks.min(axis=(1, 3)) == blocks.max(axis=(1, 3))))      # constant per block
    for g in range(3):                                                      # each gate its own 95 %
        kept = M[g * 64:(g + 1) * 64].reshape(16, 4, 24, 4)[:, 0, :, 0].mean()
        assert abs(kept - 0.05) < 1.0 / (16 * 24) + 1e-9
    # the kept blocks are the largest-L1 ones of their gate
    l1 = np.abs(W[:64]).reshape(16, 4, 24, 4).sum(axis=(1, 3))
    keep = M[:64].reshape(16, 4, 24, 4)[:, 0, :, 0] > 0
    assert l1[keep].min() >= l1[~keep].max()


def test_prune_state_sparsifies_only_gru_weights():
    d = syn.TINY_MOL
    st = syn.make_fatchord_state(d, 0)
    pr = pruning.prune_state(st, 0.9)
    for k in st:
        if k in pruning.GRU_KEYS:
            assert pruning.block_density(pr[k]) <= 0.1 + 4 * 16 / pr[k].size + 1e-9   # int(n·z) rounding
            nz = pr[k] != 0
            np.testing.assert_array_equal(pr[k][nz], st[k][nz])
        else:
            assert pr[k] is st[k]


def test_cubic_schedule():
    assert pruning.sparsity_at(0, 1000, 200_000, 0.95) == 0.0
    assert pruning.sparsity_at(1000 + 200_000, 1000, 200_000, 0.95) == 0.95
    z = pruning.sparsity_at(1000 + 100_000, 1000, 200_000, 0.95)
    assert abs(z - 0.95 * (1 - 0.5 ** 3)) < 1e-12
