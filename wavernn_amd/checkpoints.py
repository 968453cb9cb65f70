"""Checkpoint directory layout and the latest / named weight + optimizer pairs a reference
training loop writes (`utils/paths.py:5-71`, `utils/checkpoints.py:6-132`), for pointing such a
loop at the drop-in `WaveRNN`.  Training is outside the generation hot path:
this module is only the file contract, so existing checkpoint directories keep working.

Contract kept: the file names under `checkpoints/<id>.wavernn|.tacotron/` (`latest_weights.pyt`,
`latest_optim.pyt`, `<name>_weights.pyt`, `<name>_optim.pyt`), the rule that a pair is either
complete or absent (one file alone is an error, FileNotFoundError), restore-or-create, and
seeding a new pair from initial weights with the step counter reset.

Design (not the reference's): a pair is a `CheckpointPair` value with a `status()`; saving and
restoring are one function each over such pairs; progress goes to a `log` callable (default
`print`, silenced with `is_silent`); kinds are looked up in a table (`'voc'`, `'tts'`), so an
unknown kind raises NotImplementedError like the reference.  Optimizer state is read with
`torch.load(..., weights_only=True)` (a torch.optim state_dict is tensors, numbers and lists).
`Paths` takes `base=` and `ignore_voc` / `ignore_tts` keywords instead of reading `hp` from
`__main__` (`paths.py:44`).
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Callable, Dict, Optional, Tuple, Union

import torch

PathLike = Union[str, Path]

# model kind → (Paths attribute prefix, checkpoint directory suffix)
_KINDS: Dict[str, Tuple[str, str]] = {"voc": ("voc", "wavernn"), "tts": ("tts", "tacotron")}


class Paths:
    """Directory layout of a run: data under `data_path`, checkpoints and outputs under `base`."""

    _DATA_SUBDIRS = ("quant", "mel", "gta")

    def __init__(self, data_path: PathLike, voc_id: str, tts_id: str, *, base: Optional[PathLike] = None,
                 ignore_voc: bool = False, ignore_tts: bool = False, create: bool = True):
        self.base = Path(base if base is not None else Path.cwd()).expanduser().resolve()
        self.data = Path(data_path).expanduser().resolve()
        for sub in self._DATA_SUBDIRS:
            setattr(self, sub, self.data / sub)
        self.gta_model = self.data / f"gta_{tts_id}"
        self.attn_model = self.data / f"attn_{tts_id}"
        for kind, model_id in (("voc", voc_id), ("tts", tts_id)):
            prefix, suffix = _KINDS[kind]
            ck = self.base / "checkpoints" / f"{model_id}.{suffix}"
            setattr(self, f"{prefix}_checkpoints", ck)
            setattr(self, f"{prefix}_latest_weights", ck / "latest_weights.pyt")
            setattr(self, f"{prefix}_latest_optim", ck / "latest_optim.pyt")
            setattr(self, f"{prefix}_output", self.base / "model_outputs" / f"{model_id}.{suffix}")
            setattr(self, f"{prefix}_step", ck / "step.npy")
            setattr(self, f"{prefix}_log", ck / "log.txt")
        self.tts_attention = self.tts_checkpoints / "attention"
        self.tts_mel_plot = self.tts_checkpoints / "mel_plots"
        self._ignore = {"voc": ignore_voc, "tts": ignore_tts}
        if create:
            self.create_paths()

    def _dirs(self):
        yield from (self.data, *(getattr(self, s) for s in self._DATA_SUBDIRS))
        if not self._ignore["voc"]:
            yield from (self.voc_checkpoints, self.voc_output)
        if not self._ignore["tts"]:
            yield from (self.tts_checkpoints, self.tts_output, self.tts_attention, self.tts_mel_plot)

    def create_paths(self):
        for d in self._dirs():
            d.mkdir(parents=True, exist_ok=True)

    def get_voc_named_weights(self, name: str) -> Path:
        return checkpoint_pair("voc", self, name).weights

    def get_voc_named_optim(self, name: str) -> Path:
        return checkpoint_pair("voc", self, name).optim

    def get_tts_named_weights(self, name: str) -> Path:
        return checkpoint_pair("tts", self, name).weights

    def get_tts_named_optim(self, name: str) -> Path:
        return checkpoint_pair("tts", self, name).optim


@dataclass(frozen=True)
class CheckpointPair:
    """Weights file + optimizer file that are written and read together."""
    weights: Path
    optim: Path
    label: str                     # "latest" or "named"

    def status(self) -> str:
        """'complete', 'absent' or 'broken' (exactly one of the two files exists)."""
        present = self.weights.exists() + self.optim.exists()
        return ("absent", "broken", "complete")[present]


def checkpoint_pair(kind: str, paths: Paths, name: Optional[str] = None) -> CheckpointPair:
    if kind not in _KINDS:
        raise NotImplementedError(f"unknown checkpoint kind {kind!r}")
    ck: Path = getattr(paths, f"{_KINDS[kind][0]}_checkpoints")
    if name:
        return CheckpointPair(ck / f"{name}_weights.pyt", ck / f"{name}_optim.pyt", "named")
    return CheckpointPair(ck / "latest_weights.pyt", ck / "latest_optim.pyt", "latest")


def get_checkpoint_paths(checkpoint_type: str, paths: Paths):
    """(latest weights, latest optimizer, checkpoint directory) of a kind."""
    pair = checkpoint_pair(checkpoint_type, paths)
    return pair.weights, pair.optim, pair.weights.parent


def _write_pair(pair: CheckpointPair, model, optimizer, log: Callable[[str], None]) -> None:
    state = pair.status()
    if state == "broken":
        raise FileNotFoundError(f"{pair.label} checkpoint {pair.weights.parent} holds only one of "
                                f"{pair.weights.name} / {pair.optim.name}")
    pair.weights.parent.mkdir(parents=True, exist_ok=True)
    log(f"{'new' if state == 'absent' else 'overwriting'} {pair.label} checkpoint: {pair.weights}, {pair.optim}")
    model.save(pair.weights)
    torch.save(optimizer.state_dict(), pair.optim)


def save_checkpoint(checkpoint_type: str, paths: Paths, model, optimizer, *, name: Optional[str] = None,
                    is_silent: bool = False, log: Callable[[str], None] = print) -> None:
    """Write the latest pair and, with `name`, the named pair too.  Every pair involved is
    checked before anything is written."""
    pairs = [checkpoint_pair(checkpoint_type, paths)] + ([checkpoint_pair(checkpoint_type, paths, name)] if name else [])
    broken = [p for p in pairs if p.status() == "broken"]
    if broken:
        raise FileNotFoundError(f"{broken[0].label} checkpoint holds only one of its two files: "
                                f"{broken[0].weights.parent}")
    out = (lambda _msg: None) if is_silent else log
    for pair in pairs:
        _write_pair(pair, model, optimizer, out)


def restore_checkpoint(checkpoint_type: str, paths: Paths, model, optimizer, *, name: Optional[str] = None,
                       create_if_missing: bool = False, init_weights_path: Optional[PathLike] = None,
                       log: Callable[[str], None] = print) -> None:
    """Load the latest (or named) pair into model / optimizer (optimizer state onto the model's
    device).  A missing pair is created from the current model — first seeded from
    `init_weights_path` with its step reset — when `create_if_missing`, else FileNotFoundError."""
    pair = checkpoint_pair(checkpoint_type, paths, name)
    state = pair.status()
    if state == "complete":
        log(f"restoring {pair.label} checkpoint: {pair.weights}, {pair.optim}")
        model.load(pair.weights)
        device = next(model.parameters()).device
        optimizer.load_state_dict(torch.load(pair.optim, map_location=device, weights_only=True))
        return
    if state == "broken" or not create_if_missing:
        raise FileNotFoundError(f"no usable {pair.label} checkpoint at {pair.weights.parent} ({state})")
    if init_weights_path is not None:
        model.load(init_weights_path)
        model.step.zero_()
        log(f"seeded from {init_weights_path} (step reset)")
    save_checkpoint(checkpoint_type, paths, model, optimizer, name=name, log=log)
