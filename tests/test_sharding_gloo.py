"""Multi-process (gloo, world_size 2, CPU) tests of utterance sharding + the audio gather.

generate_many() itself needs a GPU, so the per-block generator is replaced by a deterministic
function of the global utterance index and the global row id the block starts at; what is
under test is the partition, the row-id bookkeeping (Philox keys) and the collective that
reassembles the audio on rank 0 in input order."""
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


class _RowsModel:
    """Stand-in for WaveRNN.rows_of: a "mel" is its frame count; batched → T // 10 + 1 folds."""

    @staticmethod
    def rows_of(T, batched, target, overlap):
        return T // 10 + 1 if batched else 1


def _rows_before(mels, i, batched):
    return sum(_RowsModel.rows_of(m, batched, 0, 0) for m in mels[:i])


def _worker(rank, world, port, n_items, batched, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mels = [np.zeros((1, 4, 20 + 7 * i)) for i in range(n_items)]
        calls = []

        def gen(ii, ms, r0):
            calls.append(len(ii))
            # one launch per rank: the block's first row id is the global one
            assert r0 == _rows_before([m.shape[-1] for m in mels], ii[0], batched)
            return [fake_audio(i) for i in ii]

        out = sharding.generate_sharded(_RowsModel(), mels, batched, 0, 0, False, device=torch.device("cpu"),
                                        generate_fn=gen)
        # the rank's launch carries exactly its contiguous block: the launch's row count (and so the
        # loop kernel choose_path picks, sharding.py docstring) is a function of (n, rank, world)
        block = sharding.shard_indices(n_items, rank, world)
        assert calls == ([len(block)] if block else [])
        dm = sharding.generate_sharded_deepmind(None, n_items, 5, device=torch.device("cpu"),
                                                generate_fn=lambda ii, r0: [np.arange(5) * 1000 - 32768 + i
                                                                            for i in ii])
        # one utterance's folds across the ranks: fold i "generates" fake_audio(i)[:64] (float32)
        folds = sharding.generate_sharded_folds(_RowsModel(), mels[-1], 0, 0, False, device=torch.device("cpu"),
                                                fold_fn=lambda ii: np.stack([fake_audio(i)[:64].astype(np.float32)
                                                                             for i in ii]),
                                                post_fn=lambda y: y)
        if rank == 0:
            q.put(([None if o is None else o.tolist() for o in out], [d.tolist() for d in dm],
                   [str(d.dtype) for d in dm], folds.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_items,batched", [(5, False), (2, True), (1, False), (9, True)])
def test_sharded_gather_reassembles_in_order(n_items, batched):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_items, batched, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, dm, dm_dtypes, folds = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == n_items
    for i, a in enumerate(got):
        a = np.asarray(a)
        assert a.dtype == np.float64
        np.testing.assert_array_equal(a, fake_audio(i))     # bit-exact float64
    assert dm_dtypes == ["int64"] * n_items
    for i, d in enumerate(dm):
        np.testing.assert_array_equal(d, np.arange(5) * 1000 - 32768 + i)
    n_folds = _RowsModel.rows_of(20 + 7 * (n_items - 1), True, 0, 0)
    np.testing.assert_array_equal(np.asarray(folds, np.float32),
                                  np.stack([fake_audio(i)[:64].astype(np.float32) for i in range(n_folds)]))


def test_shard_indices_partition():
    for n in (0, 1, 7, 64):
        for world in (1, 2, 3, 8):
            parts = [sharding.shard_indices(n, r, world) for r in range(world)]
            flat = [i for p in parts for i in p]
            assert flat == list(range(n))                    # contiguous blocks, in order
            assert max(map(len, parts)) - min(map(len, parts)) <= 1


class _NoiseModel(_RowsModel):
    """Stand-in model whose generate_many records the injected draws it receives (the slice of the
    whole list's [L_max][rows][K] noise for the rank's rows); hop_length as WaveRNN's."""
    hop_length = 275

    def __init__(self):
        self.got = []

    def generate_many(self, ms, save_paths, batched, target, overlap, mu_law, *, seed, row_offset, noise):
        self.got.append((row_offset, None if noise is None else np.asarray(noise).copy()))
        return [fake_audio(int(row_offset) + j) for j in range(len(ms))]


def _noise_worker(rank, world, port, batched, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = [20, 27, 34, 41, 48]
        mels = [np.zeros((1, 4, T)) for T in frames]
        rows = [_RowsModel.rows_of(T, batched, 0, 0) for T in frames]
        L = max(T * _NoiseModel.hop_length for T in frames) if not batched else 64
        noise = np.arange(L * sum(rows) * 3, dtype=np.float32).reshape(L, sum(rows), 3)
        m = _NoiseModel()
        sharding.generate_sharded(m, mels, batched, 32, 16, False, device=torch.device("cpu"), noise=noise)
        block = sharding.shard_indices(len(mels), rank, world)
        r0, n = sum(rows[:block[0]]), sum(rows[i] for i in block)
        steps = 32 + 2 * 16 if batched else max(frames[i] for i in block) * _NoiseModel.hop_length
        (row_offset, got), = m.got
        ok = row_offset == r0 and got.shape == (steps, n, 3) and np.array_equal(got, noise[:steps, r0:r0 + n])
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batched", [False, True])
def test_sharded_noise_injection_slices_the_rank_rows(batched):
    """generate_sharded(noise=): each rank's one launch receives exactly its rows' draws of the whole
    list's injected noise (global row order, steps trimmed to the rank's launch)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_noise_worker, args=(r, world, port, batched, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: True, 1: True}
