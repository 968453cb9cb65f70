"""Multi-process (gloo, world_size 2, CPU) tests of utterance sharding + the audio gather.

generate() itself needs a GPU, so the per-utterance generator is replaced by a deterministic
function of the global utterance index; what is under test is the partition and the
collective that reassembles the audio on rank 0 in input order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from wavernn_amd import sharding


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def fake_audio(i: int) -> np.ndarray:
    """float64 audio with bits float32 cannot hold: the gather must not round it"""
    rng = np.random.default_rng(100 + i)
    a = rng.uniform(-1, 1, size=1000 + 37 * i)
    assert not np.array_equal(a, a.astype(np.float32).astype(np.float64))
    return a


def _worker(rank, world, port, n_items, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = sharding.generate_sharded(None, [None] * n_items, False, 0, 0, False, device=torch.device("cpu"),
                                        generate_fn=lambda i, m: fake_audio(i))
        if rank == 0:
            q.put([None if o is None else o.tolist() for o in out])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_items", [5, 2, 1])
def test_sharded_gather_reassembles_in_order(n_items):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_items, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == n_items
    for i, a in enumerate(got):
        a = np.asarray(a)
        assert a.dtype == np.float64
        np.testing.assert_array_equal(a, fake_audio(i))     # bit-exact float64


def test_shard_indices_partition():
    for n in (0, 1, 7, 64):
        for world in (1, 2, 3, 8):
            parts = [sharding.shard_indices(n, r, world) for r in range(world)]
            flat = sorted(i for p in parts for i in p)
            assert flat == list(range(n))
