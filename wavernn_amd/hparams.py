"""Hyper-parameter pseudo-module (the reference's utils/__init__.py:40-92 `hparams`).

`hparams.configure(path)` copies the attributes of a Python hparams file (the reference's
hparams.py format) once; reading an attribute before configuring raises.  The vocoder /
DSP defaults the generation path needs (hparams.py:20-60) are available through
`DEFAULTS` for callers that have no hparams file."""
from __future__ import annotations

import re
from importlib.util import module_from_spec, spec_from_file_location
from pathlib import Path
from typing import Union

DEFAULTS = dict(
    sample_rate=22050, n_fft=2048, num_mels=80, hop_length=275, win_length=1100, fmin=40,
    min_level_db=-100, ref_level_db=20, bits=9, mu_law=True, peak_norm=False,
    voc_mode='MOL', voc_upsample_factors=(5, 5, 11), voc_rnn_dims=512, voc_fc_dims=512,
    voc_compute_dims=128, voc_res_out_dims=128, voc_res_blocks=10, voc_pad=2,
    voc_gen_batched=True, voc_target=11_000, voc_overlap=550, voc_gen_at_checkpoint=5,
)


class HParams:
    def __init__(self):
        object.__setattr__(self, "_configured", False)

    def __getattr__(self, item):
        if not object.__getattribute__(self, "_configured"):
            raise AttributeError("HParams not configured yet. Call hparams.configure()")
        raise AttributeError(item)

    def is_configured(self) -> bool:
        return object.__getattribute__(self, "_configured")

    def configure(self, path: Union[str, Path, None] = None, **overrides):
        """Load a hparams .py file (or the built-in DEFAULTS when path is None)."""
        if self.is_configured():
            raise RuntimeError("Cannot reconfigure hparams!")
        values = dict(DEFAULTS)
        if path is not None:
            p = Path(path).expanduser()
            if not p.exists():
                raise FileNotFoundError(f"Could not find hparams file {p}")
            if p.suffix != ".py":
                raise ValueError("`path` must be a python file")
            spec = spec_from_file_location("hparams", p)
            m = module_from_spec(spec)
            spec.loader.exec_module(m)
            magic = re.compile(r"^__.+__$")
            values.update({k: v for k, v in vars(m).items() if not magic.match(k)})
        values.update(overrides)
        for k, v in values.items():
            if k in ("configure", "is_configured"):
                raise AttributeError(f"hparams file cannot define {k}")
            object.__setattr__(self, k, v)
        object.__setattr__(self, "_configured", True)
        return self


hparams = HParams()
