"""Multi-utterance drop-in entry points on the MI355X.

* `WaveRNN.generate_many(mels)` runs several utterances (or all their folds) as the rows of ONE
  loop launch; under Philox each utterance equals its own `generate(mel, row_offset=<first row>)`
  (row-keyed draws, the same kernel) within the MoL tolerance used between launches of different
  shapes (2·MOL_TOL): the launch shape picks the loop kernel (one-row XCD kernel up to 8 MoL rows,
  the many-row one from 9) and the rocBLAS terms GEMM over all utterances' frames picks its tiling
  by shape, so the conditioning terms may differ in the last bit; the deepmind rows (no conditioning) and RAW
  labels are compared exactly.
* Config 4's shape: 8 utterances of the rnn-896 block-sparse model in one launch of the sparse
  XCD kernel vs 8 separate calls.  Config 5's: 32 deepmind rows vs 32 single-row calls.
* A loop handle that ran the many-row kernel must still run the one-row kernel afterwards
  (the one-row kernel's hop buffer was allocated only with the member counters).
Reference behaviour being batched: gen_wavernn.py:11-35 (one generate() per utterance),
models/fatchord_version.py:169-264, models/deepmind_version.py:75-165."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf

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


def _close(a, b, what):
    assert a.dtype == np.float64 and a.shape == b.shape, what
    err = np.abs(a - b).max()
    print(f"{what}: max |Δ| {err:.3g}")
    assert err <= 2 * gf.MOL_TOL, (what, err)


def _mels(d, frames, seed0):
    return [torch.from_numpy(syn.make_mel(d.feat_dims, T, seed0 + i))[None] for i, T in enumerate(frames)]


@pytest.mark.parametrize("frames", [(30, 30, 30), (30, 41, 25, 22)])
def test_generate_many_unbatched_equals_single_calls(frames):
    d = syn.DEFAULT_MOL
    m = _model(d, 3)
    mels = _mels(d, frames, 50)
    got = m.generate_many(mels, None, False, 11000, 550, True, seed=123)
    path_many = m.loop_handle().info["last_path"]
    assert path_many == 5                       # rows <= 8: one row per XCD
    for i, mel in enumerate(mels):
        ref = m.generate(mel, None, False, 11000, 550, True, seed=123, row_offset=i, verbose=False)
        assert m.loop_handle().info["last_path"] == path_many
        _close(got[i], ref, f"utterance {i}")


def test_generate_many_batched_folds_keyed_by_global_row():
    d = syn.DEFAULT_MOL
    m = _model(d, 4)
    mels = _mels(d, (81, 60), 70)                # 4 + 3 folds at target 6000 / overlap 300: 7 rows
    target, overlap = 6000, 300
    rows = [m.rows_of(x.shape[-1], True, target, overlap) for x in mels]
    got = m.generate_many(mels, None, True, target, overlap, True, seed=5, row_offset=10)
    assert m.loop_handle().info["last_path"] == 5
    r0 = 10
    for i, mel in enumerate(mels):
        ref = m.generate(mel, None, True, target, overlap, True, seed=5, row_offset=r0, verbose=False)
        _close(got[i], ref, f"utterance {i}")
        r0 += rows[i]


def test_generate_many_sparse896_eight_utterances():
    """Config 4's per-GPU shape: 8 utterances of the 95 % 4x4 block-sparse rnn-896 model."""
    d = syn.SPARSE896_MOL
    m = _model(d, 0, prune=0.95)
    mels = _mels(d, [24] * 8, 90)
    got = m.generate_many(mels, None, False, 11000, 550, True, seed=31)
    h = m.loop_handle()
    assert h.info["last_path"] == 6 and h.info["sparse_blocks"] > 0, h.info
    for i, mel in enumerate(mels):
        ref = m.generate(mel, None, False, 11000, 550, True, seed=31, row_offset=i, verbose=False)
        _close(got[i], ref, f"sparse utterance {i}")


def test_deepmind_batch32_equals_single_rows():
    """Config 5's per-GPU shape: 32 deepmind utterances in one launch vs each row alone."""
    from wavernn_amd.deepmind_version import WaveRNN as DM
    d = syn.DEFAULT_DM
    m = DM(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_deepmind_state(d, 1).items()})
    out, coarse, fine = m.generate(400, batch=32, seed=17)
    assert m.loop_handle().info["last_path"] == 8
    for b in range(32):
        o, c, f = m.generate(400, seed=17, row_offset=b)
        assert np.array_equal(o, out[b]) and np.array_equal(c, coarse[b]) and np.array_equal(f, fine[b]), b


def test_one_row_kernel_after_many_row_kernel_on_one_handle():
    """B=10 (many-row kernel) then B=1 (one-row kernel) on ONE handle."""
    from wavernn_amd.loop import FatchordLoop
    d = syn.DEFAULT_MOL
    st = syn.make_fatchord_state(d, 2)
    L = 600
    mels, aux = syn.make_conditioning(10, L, d.feat_dims, d.res_out_dims, 8)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)

    def fresh():
        lp = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
        lp.set_weights(st)
        return lp

    loop = fresh()
    loop.generate(cond, seed=3)
    assert loop.info["last_path"] == 7
    one = cond[:, :1].contiguous()
    y1, _ = loop.generate(one, seed=3)
    assert loop.info["last_path"] == 5
    other = fresh()
    y2, _ = other.generate(one, seed=3)
    assert torch.equal(y1, y2)
    loop.close()
    other.close()


def test_generate_many_raw_labels_exact():
    """RAW (bits) rows of one launch vs single calls: the mu-law-decoded waveforms, i.e. the
    integer labels, identical (config 1's model; the many-row kernel's softmax head)."""
    d = syn.DEFAULT_RAW
    m = _model(d, 6)
    mels = _mels(d, (25, 28), 120)
    got = m.generate_many(mels, None, False, 11000, 550, True, seed=8)
    for i, mel in enumerate(mels):
        ref = m.generate(mel, None, False, 11000, 550, True, seed=8, row_offset=i, verbose=False)
        assert np.array_equal(got[i], ref), i
