"""Utterance sharding across GPUs (one process per GPU, torch.distributed).

The reference generates one utterance at a time on one device (gen_wavernn.py:11-35 loops
over the test set).  Utterances are independent, so the MI355X path shards them: rank r takes a
contiguous block of the list (block sizes differ by at most one) and vocodes the whole block as
the rows of ONE persistent-kernel launch (`WaveRNN.generate_many`; deepmind: `generate(batch=)`).
Each loop row's sampler draws are keyed by its GLOBAL row id (Philox (seed, row)), so every
utterance sees the same random draws whatever the number of GPUs.  What the GPU count does change
is the SHAPE of each rank's launch (its row count), and with it the kernel the C-ABI picks
(`choose_path`, capi.cpp: MoL rnn 512 runs fatchord_xcd_kernel up to 8 rows and
fatchord_xcdm_kernel from 9; RAW and deepmind one kernel at every row count) and the tiling the
frame-rate terms GEMM gets.  So the promise is: deepmind outputs bit-identical across world sizes;
RAW labels identical in every test so far (the terms are rounded differently, so a label exactly at
a tie could flip); MoL samples equal within the MoL parity tolerance (2·MOL_TOL in
tests/test_gpu_many.py), not bit for bit — the same contract as generate_many vs single calls.  The only collective is the final gather of
finished audio to rank 0 (RCCL over xGMI under the "nccl" backend; gloo on CPU for tests) —
there is no exchange inside the sample loop.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist


def world_rank(group=None):
    """(world size, rank) of the group; (1, 0) without an initialised process group (a single
    GPU runs the same entry points with no collective)."""
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def shard_indices(n_items: int, rank: int, world: int) -> List[int]:
    """Contiguous block of rank `rank`: items [rank·n // world, (rank + 1)·n // world)."""
    return list(range(rank * n_items // world, (rank + 1) * n_items // world))


def gather_audio(local: Dict[int, np.ndarray], n_items: int, device: torch.device,
                 group=None) -> Optional[List[np.ndarray]]:
    """Collect {global index: float64 audio} from every rank on rank 0, in global order.

    Shapes differ per utterance, so each rank packs its outputs into a [n_slots, L_max] float64
    tensor plus an int64 [n_slots, 2] (index, length) table; two all-gathers move them.  The
    audio travels as the float64 generate() returns (RCCL and gloo move float64 natively), so
    rank 0's list is bit-identical to what each rank's generate() produced."""
    world, rank = world_rank(group)
    if world == 1 and not dist.is_initialized():
        out = [None] * n_items
        for idx, audio in local.items():
            out[idx] = np.asarray(audio, dtype=np.float64)
        return out
    n_slots = (n_items + world - 1) // world
    lens = torch.tensor([max((len(v) for v in local.values()), default=0)], dtype=torch.int64, device=device)
    dist.all_reduce(lens, op=dist.ReduceOp.MAX, group=group)
    L = int(lens.item())
    data = torch.zeros(n_slots, max(L, 1), dtype=torch.float64, device=device)
    meta = torch.full((n_slots, 2), -1, dtype=torch.int64, device=device)
    for s, (idx, audio) in enumerate(sorted(local.items())):
        data[s, :len(audio)] = torch.as_tensor(np.asarray(audio, dtype=np.float64), device=device)
        meta[s, 0], meta[s, 1] = idx, len(audio)
    if dist.get_backend(group) == "nccl":
        all_data = torch.empty(world * n_slots, data.shape[1], dtype=data.dtype, device=device)
        all_meta = torch.empty(world * n_slots, 2, dtype=meta.dtype, device=device)
        dist.all_gather_into_tensor(all_data, data, group=group)
        dist.all_gather_into_tensor(all_meta, meta, group=group)
    else:
        dl = [torch.empty_like(data) for _ in range(world)]
        ml = [torch.empty_like(meta) for _ in range(world)]
        dist.all_gather(dl, data, group=group)
        dist.all_gather(ml, meta, group=group)
        all_data, all_meta = torch.cat(dl), torch.cat(ml)
    if rank != 0:
        return None
    out: List[Optional[np.ndarray]] = [None] * n_items
    all_data = all_data.cpu().numpy()
    for row, (idx, n) in enumerate(all_meta.cpu().numpy()):
        if idx >= 0:
            out[int(idx)] = all_data[row, :int(n)].copy()
    return out  # type: ignore[return-value]


def generate_sharded(model, mels: Sequence, batched: bool, target: int, overlap: int, mu_law: bool,
                     base_seed: int = 0, device: Optional[torch.device] = None, group=None,
                     generate_fn: Optional[Callable] = None, noise=None) -> Optional[List[np.ndarray]]:
    """Generate every mel in `mels` across the process group; rank 0 returns the list of
    float64 waveforms in input order, other ranks return None.

    `noise` (optional, parity testing): the injected draws of the WHOLE list, [L_max][rows][K]
    in global row order (generate_many's layout on one GPU); each rank passes its rows' slice.

    A rank runs its block through ONE `generate_many` launch, seeded `base_seed` with its first
    loop row at the global row id of its first utterance (every rank knows every mel's row
    count from its length), so the result equals `model.generate_many(mels, seed=base_seed)` on
    one GPU — MoL within the parity tolerance, since a rank's launch shape (and so its kernel,
    module docstring) depends on the world size.  `generate_fn(indices, mels, row_offset)` replaces the generation (host tests)."""
    world, rank = world_rank(group)
    if device is None:
        device = next(model.parameters()).device
    idx = shard_indices(len(mels), rank, world)
    rows = [model.rows_of(np.shape(m)[-1], batched, target, overlap) for m in mels]
    row0 = int(sum(rows[:idx[0]])) if idx else 0
    nz = None
    if noise is not None and idx:
        n_rows = int(sum(rows[i] for i in idx))
        steps = max((target + 2 * overlap) if batched else np.shape(mels[i])[-1] * model.hop_length for i in idx)
        nz = np.asarray(noise)[:steps, row0:row0 + n_rows]
    gen = generate_fn or (lambda ii, ms, r0: model.generate_many(ms, None, batched, target, overlap, mu_law,
                                                                  seed=base_seed, row_offset=r0, noise=nz))
    outs = gen(idx, [mels[i] for i in idx], row0) if idx else []
    return gather_audio(dict(zip(idx, outs)), len(mels), device, group)


def generate_sharded_deepmind(model, n_utterances: int, seq_len: int, base_seed: int = 0,
                              device: Optional[torch.device] = None, group=None,
                              generate_fn: Optional[Callable] = None) -> Optional[List[np.ndarray]]:
    """deepmind_version.generate(seq_len) for n_utterances independent utterances across the
    process group (BASELINE config 5: 256 over 8 GPUs): rank r runs its contiguous block as the
    rows of one `generate(batch=...)` launch keyed by the global utterance index, rank 0 returns
    the int64 outputs (coarse·256 + fine − 2^15) in utterance order.  Outputs travel as float64
    (exact: |v| ≤ 2^15)."""
    world, rank = world_rank(group)
    if device is None:
        device = next(model.parameters()).device
    idx = shard_indices(n_utterances, rank, world)

    def _gen(ii, r0):
        out, _, _ = model.generate(seq_len, batch=len(ii), seed=base_seed, row_offset=r0)
        return list(np.asarray(out).reshape(len(ii), seq_len))

    outs = (generate_fn or _gen)(idx, idx[0]) if idx else []
    got = gather_audio({i: np.asarray(o, dtype=np.float64) for i, o in zip(idx, outs)}, n_utterances, device, group)
    return None if got is None else [g.astype(np.int64) for g in got]


def generate_sharded_folds(model, mel, target: int, overlap: int, mu_law: bool, base_seed: int = 0,
                           device: Optional[torch.device] = None, group=None,
                           fold_fn: Optional[Callable] = None, post_fn: Optional[Callable] = None
                           ) -> Optional[np.ndarray]:
    """ONE long utterance's fold-batched generate() (fatchord_version.py:169-264 with
    batched=True; SURVEY.md §8(e): "the 60 s single-utterance case can shard folds across GPUs")
    over the process group: rank r runs the contiguous block of folds shard_indices(folds, r, world)
    as the rows of one loop launch keyed by the GLOBAL fold index (Philox row = fold), the fold
    outputs are all-gathered (float32 carried as float64: exact) and rank 0 runs the float64
    cross-fade / unfold / fade on the device.  Rank 0 returns the waveform, other ranks None; it
    equals model.generate(mel, None, True, target, overlap, mu_law, seed=base_seed) up to the
    MoL tolerance between launches of different shapes (RAW labels exactly).
    fold_fn(fold_indices) -> [n][steps] and post_fn([folds][steps] float32) -> waveform replace the
    device work (host tests)."""
    from . import condition
    world, rank = world_rank(group)
    if fold_fn is None:
        if device is None:
            device = next(model.parameters()).device
        # the frame-rate inputs only (mel + MelResNet output: kilobytes), then the loop entry for
        # this rank's folds — the same conditioning-terms route as generate(batched=True), never
        # the whole utterance's per-sample records on every rank
        mel_f, aux, wave_len = model.frames(mel)
        spec = model._upsample_spec()
        n_folds = model.rows_of(np.shape(mel)[-1], True, target, overlap)
        mu = mu_law if model.mode == 'RAW' else False

        def fold_fn(ii):
            y, _ = model.loop_handle().generate_frames(spec, mel_f, aux, target, overlap, seed=base_seed,
                                                       row_offset=ii[0], rows=(ii[0], len(ii)))
            return y.cpu().numpy()

        def post_fn(y_all):
            y = torch.from_numpy(np.ascontiguousarray(y_all, dtype=np.float32)).to(device)
            return condition.postprocess(y, True, overlap, mu, model.n_classes, wave_len,
                                         20 * model.hop_length).cpu().numpy()
    else:
        n_folds = model.rows_of(np.shape(mel)[-1], True, target, overlap)
    idx = shard_indices(n_folds, rank, world)
    local = fold_fn(idx) if idx else np.zeros((0, 0), np.float32)
    got = gather_audio({i: np.asarray(local[j], dtype=np.float64) for j, i in enumerate(idx)}, n_folds, device, group)
    if got is None:
        return None
    return post_fn(np.stack(got).astype(np.float32))
