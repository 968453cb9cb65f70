"""wrnn_generate_frames_rows: a block of a launch's rows (one utterance's folds on one GPU of a
node, sharding.generate_sharded_folds) equals those rows of the whole launch, keyed by their
global row id.  RAW labels exactly (the many-row kernel at every row count); MoL within the
parity tolerance — a different row count can pick the other XCD kernel, and the rocBLAS terms
GEMM over the block's records (the per-sample fallback, WRNN_NO_FRAME_TERMS=1: the launch's
records compacted to the block's rows) tiles by its row count (observed: not bit-identical at
15 of 16 rows on the same kernel)."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(d, seed):
    from wavernn_amd.fatchord_version import WaveRNN
    m = WaveRNN(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, seed).items()})
    return m


@pytest.mark.parametrize("mode", ["MOL", "RAW"])
@pytest.mark.parametrize("frames", [True, False])
def test_frame_rows_block_equals_whole_launch(mode, frames, monkeypatch):
    if not frames:
        monkeypatch.setenv("WRNN_NO_FRAME_TERMS", "1")
    d = syn.DEFAULT_MOL if mode == "MOL" else syn.DEFAULT_RAW
    m = _model(d, 4)
    mel = torch.from_numpy(syn.make_mel(d.feat_dims, 120, 31))[None]
    mel_f, aux, _ = m.frames(mel)
    spec = m._upsample_spec()
    loop = m.loop_handle()
    target, overlap = 2000, 100
    full, lab_full = loop.generate_frames(spec, mel_f, aux, target, overlap, seed=11, want_labels=mode == "RAW")
    n = full.shape[0]
    assert n >= 12
    for r0, cnt in ((0, n), (2, 5), (n - 3, 3), (1, n - 1)):
        y, lab = loop.generate_frames(spec, mel_f, aux, target, overlap, seed=11, row_offset=r0,
                                      want_labels=mode == "RAW", rows=(r0, cnt))
        assert y.shape == (cnt, full.shape[1])
        if mode == "RAW":
            assert torch.equal(lab, lab_full[r0:r0 + cnt]), (r0, cnt)
        else:
            assert (y - full[r0:r0 + cnt]).abs().max().item() <= gf.MOL_TOL, (r0, cnt)
    with pytest.raises(ValueError):
        loop.generate_frames(spec, mel_f, aux, target, overlap, rows=(n - 1, 2))
