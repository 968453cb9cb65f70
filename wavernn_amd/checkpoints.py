"""Checkpoint paths and the latest/named checkpoint writer of the reference training loop.

Mirrors the caller-facing contract of `utils/paths.py:5-71` (`Paths`) and
`utils/checkpoints.py:6-132` (`get_checkpoint_paths`, `save_checkpoint`,
`restore_checkpoint`), so a reference training script that checkpoints a vocoder can point at
the drop-in `WaveRNN` unchanged.  Same directory layout and file names
(`checkpoints/<voc_id>.wavernn/latest_weights.pyt`, `<name>_weights.pyt` …), same "both or
neither file exists" rule, same error types.

Differences, all on the safe side:
  * `Paths` takes `base=` (the reference derives it from its own install directory) and the
    `ignore_voc` / `ignore_tts` switches as keywords instead of importing `hp` from `__main__`
    (`paths.py:44`).
  * `checkpoint_type` is compared with `==`, not `is` (`checkpoints.py:15,19` relies on string
    interning).
  * optimizer state is read with `torch.load(..., weights_only=True)`: a checkpoint never
    executes code (a plain `torch.optim` state_dict is tensors, numbers and lists, which the
    safe loader accepts).
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Optional, Union

import torch


class Paths:
    """Data / vocoder / TTS paths (`utils/paths.py:5-71`)."""

    def __init__(self, data_path: Union[str, Path], voc_id: str, tts_id: str, *,
                 base: Union[str, Path, None] = None, ignore_voc: bool = False, ignore_tts: bool = False,
                 create: bool = True):
        self.base = Path(base if base is not None else Path.cwd()).expanduser().resolve()

        self.data = Path(data_path).expanduser().resolve()
        self.quant = self.data / 'quant'
        self.mel = self.data / 'mel'
        self.gta = self.data / 'gta'
        self.gta_model = self.data / f'gta_{tts_id}'
        self.attn_model = self.data / f'attn_{tts_id}'

        self.voc_checkpoints = self.base / 'checkpoints' / f'{voc_id}.wavernn'
        self.voc_latest_weights = self.voc_checkpoints / 'latest_weights.pyt'
        self.voc_latest_optim = self.voc_checkpoints / 'latest_optim.pyt'
        self.voc_output = self.base / 'model_outputs' / f'{voc_id}.wavernn'
        self.voc_step = self.voc_checkpoints / 'step.npy'
        self.voc_log = self.voc_checkpoints / 'log.txt'

        self.tts_checkpoints = self.base / 'checkpoints' / f'{tts_id}.tacotron'
        self.tts_latest_weights = self.tts_checkpoints / 'latest_weights.pyt'
        self.tts_latest_optim = self.tts_checkpoints / 'latest_optim.pyt'
        self.tts_output = self.base / 'model_outputs' / f'{tts_id}.tacotron'
        self.tts_step = self.tts_checkpoints / 'step.npy'
        self.tts_log = self.tts_checkpoints / 'log.txt'
        self.tts_attention = self.tts_checkpoints / 'attention'
        self.tts_mel_plot = self.tts_checkpoints / 'mel_plots'

        self._ignore_voc, self._ignore_tts = ignore_voc, ignore_tts
        if create:
            self.create_paths()

    def create_paths(self):
        for d in (self.data, self.quant, self.mel, self.gta):
            os.makedirs(d, exist_ok=True)
        if not self._ignore_voc:
            os.makedirs(self.voc_checkpoints, exist_ok=True)
            os.makedirs(self.voc_output, exist_ok=True)
        if not self._ignore_tts:
            for d in (self.tts_checkpoints, self.tts_output, self.tts_attention, self.tts_mel_plot):
                os.makedirs(d, exist_ok=True)

    def get_tts_named_weights(self, name):
        return self.tts_checkpoints / f'{name}_weights.pyt'

    def get_tts_named_optim(self, name):
        return self.tts_checkpoints / f'{name}_optim.pyt'

    def get_voc_named_weights(self, name):
        return self.voc_checkpoints / f'{name}_weights.pyt'

    def get_voc_named_optim(self, name):
        return self.voc_checkpoints / f'{name}_optim.pyt'


def get_checkpoint_paths(checkpoint_type: str, paths: Paths):
    """(latest weights, latest optimizer, checkpoint dir) for 'voc' or 'tts'
    (`utils/checkpoints.py:6-26`)."""
    if checkpoint_type == 'tts':
        return paths.tts_latest_weights, paths.tts_latest_optim, paths.tts_checkpoints
    if checkpoint_type == 'voc':
        return paths.voc_latest_weights, paths.voc_latest_optim, paths.voc_checkpoints
    raise NotImplementedError


def _named(checkpoint_path: Path, name: str):
    return {'w': checkpoint_path / f'{name}_weights.pyt', 'o': checkpoint_path / f'{name}_optim.pyt'}


def save_checkpoint(checkpoint_type: str, paths: Paths, model, optimizer, *,
                    name: Optional[str] = None, is_silent: bool = False):
    """Always rewrites the latest pair; also writes `<name>_{weights,optim}.pyt` when `name` is
    given (`utils/checkpoints.py:29-76`).  A pair with exactly one file present is broken and
    raises FileNotFoundError before anything is written."""
    weights_path, optim_path, checkpoint_path = get_checkpoint_paths(checkpoint_type, paths)

    def write(path_dict, is_named):
        s = 'named' if is_named else 'latest'
        n = sum(p.exists() for p in path_dict.values())
        if n not in (0, 2):
            raise FileNotFoundError(f'We expected either both or no files in the {s} checkpoint to '
                                    'exist, but instead we got exactly one!')
        if n == 0:
            if not is_silent:
                print(f'Creating {s} checkpoint...')
            for p in path_dict.values():
                p.parent.mkdir(parents=True, exist_ok=True)
        elif not is_silent:
            print(f'Saving to existing {s} checkpoint...')
        if not is_silent:
            print(f'Saving {s} weights: {path_dict["w"]}')
        model.save(path_dict['w'])
        if not is_silent:
            print(f'Saving {s} optimizer state: {path_dict["o"]}')
        torch.save(optimizer.state_dict(), path_dict['o'])

    write({'w': weights_path, 'o': optim_path}, False)
    if name:
        write(_named(checkpoint_path, name), True)


def restore_checkpoint(checkpoint_type: str, paths: Paths, model, optimizer, *,
                       name: Optional[str] = None, create_if_missing: bool = False,
                       init_weights_path: Union[str, Path, None] = None):
    """Loads the latest (or named) pair into `model` / `optimizer`; with `create_if_missing`,
    optionally seeds the model from `init_weights_path` (step reset to 0) and writes the pair
    (`utils/checkpoints.py:79-132`).  Missing pair without `create_if_missing` raises
    FileNotFoundError.  The optimizer state lands on the model's device, as in the reference."""
    weights_path, optim_path, checkpoint_path = get_checkpoint_paths(checkpoint_type, paths)
    if name:
        path_dict, s = _named(checkpoint_path, name), 'named'
    else:
        path_dict, s = {'w': weights_path, 'o': optim_path}, 'latest'

    if sum(p.exists() for p in path_dict.values()) == 2:
        print(f'Restoring from {s} checkpoint...')
        print(f'Loading {s} weights: {path_dict["w"]}')
        model.load(path_dict['w'])
        print(f'Loading {s} optimizer state: {path_dict["o"]}')
        device = next(model.parameters()).device
        optimizer.load_state_dict(torch.load(path_dict['o'], map_location=device, weights_only=True))
    elif create_if_missing:
        if init_weights_path is not None:
            model.load(init_weights_path)
            model.step *= 0
            print(f'Initializing with weights at: {init_weights_path}')
        save_checkpoint(checkpoint_type, paths, model, optimizer, name=name, is_silent=False)
    else:
        raise FileNotFoundError(f'The {s} checkpoint could not be found!')
