"""generate_sharded under the "nccl" backend (RCCL) on the GPU box: world_size 1, one process,
127.0.0.1 rendezvous.  The gathered float64 audio (one generate_many launch per rank) equals
each utterance's own generate() under the same Philox keying by global row id, within the MoL
tolerance between launches of different shapes (tests/test_gpu_many.py); the deepmind variant's
integer outputs bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from wavernn_amd import sharding
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_generate_sharded_nccl_world1():
    from wavernn_amd.fatchord_version import WaveRNN
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        d = syn.DEFAULT_MOL
        m = WaveRNN(**d.ctor_kwargs()).to(dev)
        m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, 3).items()})
        mels = [torch.from_numpy(syn.make_mel(d.feat_dims, T, 10 + T))[None] for T in (30, 41, 25)]
        got = sharding.generate_sharded(m, mels, False, 11000, 550, True, base_seed=77, device=dev)
        assert dist.get_backend() == "nccl" and len(got) == 3
        for i, mel in enumerate(mels):
            ref = m.generate(mel, None, False, 11000, 550, True, seed=77, row_offset=i, verbose=False)
            assert got[i].dtype == np.float64 and got[i].shape == ref.shape
            assert np.abs(got[i] - ref).max() <= 2e-5, i
        # one utterance's folds sharded (at world 1: every fold on this rank) = generate(batched=True)
        mel = torch.from_numpy(syn.make_mel(d.feat_dims, 60, 99))[None]
        wav = sharding.generate_sharded_folds(m, mel, 3000, 150, True, base_seed=5, device=dev)
        ref = m.generate(mel, None, True, 3000, 150, True, seed=5, verbose=False)
        assert wav.dtype == np.float64 and wav.shape == ref.shape and np.abs(wav - ref).max() <= 2e-5
        from wavernn_amd.deepmind_version import WaveRNN as DM
        dd = syn.DEFAULT_DM
        dm = DM(**dd.ctor_kwargs()).to(dev)
        dm.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_deepmind_state(dd, 2).items()})
        got = sharding.generate_sharded_deepmind(dm, 5, 300, base_seed=9, device=dev)
        assert len(got) == 5
        for i in range(5):
            ref, _, _ = dm.generate(300, seed=9, row_offset=i)
            assert got[i].dtype == np.int64 and np.array_equal(got[i], ref), i
    finally:
        dist.destroy_process_group()
