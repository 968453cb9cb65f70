"""Block-sparse GRU pruning (BASELINE config 4: rnn_dims 896, 4x4 blocks, 95 % sparsity).

The reference prunes element-wise (notebooks/Pruning - Scratchpad.ipynb, PruneMask: per-gate
split `splits={'GRU': 3}` :54, W_ih and W_hh both pruned when `prune_rnn_input` :59, per-gate
threshold `sorted_abs[k]` with `k = int(numel · z)` and mask `|W| >= threshold` :92-108, cubic
schedule z = Z·(1 − (1 − (t − t0)/S)^3) :145).  SURVEY.md §8 a16 defines the block variant this
build targets: the same per-gate rule applied to the L1 norms of 4x4 blocks, so the zeros come
in whole blocks that the multi-row kernel skips (capi.cpp detects them at wrnn_set_weights).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

GRU_KEYS = ("rnn1.weight_ih_l0", "rnn1.weight_hh_l0", "rnn2.weight_ih_l0", "rnn2.weight_hh_l0")


def sparsity_at(t: float, t0: float, steps: float, target: float) -> float:
    """Cubic schedule (Pruner.update_sparsity), clamped to [0, target]."""
    z = target * (1.0 - (1.0 - (t - t0) / steps) ** 3)
    return float(min(max(z, 0.0), target))


def block_mask(W: np.ndarray, z: float, block: int = 4, splits: int = 3) -> np.ndarray:
    """0/1 mask of W's (block x block) blocks, per gate slice: blocks whose L1 norm is below
    the k-th smallest (k = int(n_blocks · z)) are zeroed; ties at the threshold are kept."""
    rows, cols = W.shape
    if rows % (splits * block) or cols % block:
        raise ValueError(f"{W.shape} does not tile into {splits} gate slices of {block}x{block} blocks")
    gs = rows // splits
    out = np.empty_like(W, dtype=np.float32)
    for g in range(splits):
        Wg = W[g * gs:(g + 1) * gs]
        l1 = np.abs(Wg).reshape(gs // block, block, cols // block, block).sum(axis=(1, 3))
        k = int(l1.size * z)
        thr = np.sort(l1.reshape(-1))[min(k, l1.size - 1)]
        keep = (l1 >= thr).astype(np.float32)
        out[g * gs:(g + 1) * gs] = np.repeat(np.repeat(keep, block, axis=0), block, axis=1)
    return out


def prune_state(state: Dict[str, np.ndarray], z: float = 0.95, block: int = 4) -> Dict[str, np.ndarray]:
    """Copy of a fatchord state_dict with every GRU weight matrix block-pruned to sparsity z."""
    out = dict(state)
    for k in GRU_KEYS:
        W = np.asarray(state[k], dtype=np.float32)
        out[k] = (W * block_mask(W, z, block)).astype(np.float32)
    return out


def block_density(W: np.ndarray, block: int = 4) -> float:
    """Fraction of (block x block) blocks of W with any nonzero entry."""
    r, c = W.shape
    nz = np.abs(W[: r - r % block, : c - c % block]).reshape(r // block, block, c // block, block).sum(axis=(1, 3))
    return float((nz > 0).mean())
