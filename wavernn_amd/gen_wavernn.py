"""Vocoder CLI on the MI355X path — the reference's gen_wavernn.py:68-150 flags.

    python -m wavernn_amd.gen_wavernn -f mel.npy [-b|-u] [-t T] [-o O] [-w weights.pyt]
                                      [--hp_file hparams.py] [--out_dir DIR]

Mel input is a normalised (n_mels, n_hops) .npy in [0, 1] (checked like gen_wavernn.py:48-57).
The test-set mode and wav input need the training data pipeline / librosa feature
extraction, which are out of scope; they raise.  (wavernn_amd.dsp
.load_wav reads wavs for other callers, but unlike the reference's librosa.load it does not
resample: a file at another rate than hp.sample_rate raises.)
"""
from __future__ import annotations

import argparse
from pathlib import Path

import numpy as np
import torch

from .hparams import HParams


def build_model(hp, device):
    from .fatchord_version import WaveRNN
    return WaveRNN(rnn_dims=hp.voc_rnn_dims, fc_dims=hp.voc_fc_dims, bits=hp.bits, pad=hp.voc_pad,
                   upsample_factors=hp.voc_upsample_factors, feat_dims=hp.num_mels,
                   compute_dims=hp.voc_compute_dims, res_out_dims=hp.voc_res_out_dims,
                   res_blocks=hp.voc_res_blocks, hop_length=hp.hop_length, sample_rate=hp.sample_rate,
                   mode=hp.voc_mode).to(device)


def load_mel(path: Path, n_mels: int) -> np.ndarray:
    if path.suffix != ".npy":
        raise ValueError(f"Expected a .npy mel (wav feature extraction is out of scope), got {path.suffix}")
    mel = np.load(path, allow_pickle=False)
    if mel.ndim != 2 or mel.shape[0] != n_mels:
        raise ValueError(f"Expected a numpy array shaped (n_mels, n_hops), but got {mel.shape}!")
    if mel.max() >= 1.01 or mel.min() <= -0.01:
        raise ValueError(f"Expected spectrogram range in [0,1] but was instead [{mel.min()}, {mel.max()}]")
    return mel


def main(argv=None):
    ap = argparse.ArgumentParser(description="Generate WaveRNN samples on MI355X")
    ap.add_argument("--batched", "-b", dest="batched", action="store_true", help="Fast Batched Generation")
    ap.add_argument("--unbatched", "-u", dest="batched", action="store_false", help="Slow Unbatched Generation")
    ap.add_argument("--target", "-t", type=int)
    ap.add_argument("--overlap", "-o", type=int)
    ap.add_argument("--file", "-f", type=str, required=True, help="mel .npy to vocode")
    ap.add_argument("--voc_weights", "-w", type=str, help="reference-format state_dict (*.pyt)")
    ap.add_argument("--hp_file", metavar="FILE", default=None)
    ap.add_argument("--out_dir", default=".")
    ap.add_argument("--seed", type=int, default=None)
    ap.set_defaults(batched=None)
    args = ap.parse_args(argv)
    hp = HParams().configure(args.hp_file)
    target = args.target if args.target is not None else hp.voc_target
    overlap = args.overlap if args.overlap is not None else hp.voc_overlap
    batched = args.batched if args.batched is not None else hp.voc_gen_batched
    if not torch.cuda.is_available():
        raise RuntimeError("the MI355X generation path needs a GPU")
    model = build_model(hp, torch.device("cuda"))
    if args.voc_weights:
        model.load(args.voc_weights)
    path = Path(args.file).expanduser()
    mel = torch.from_numpy(load_mel(path, hp.num_mels)).unsqueeze(0)
    k = model.get_step() // 1000
    tag = f"gen_batched_target{target}_overlap{overlap}" if batched else "gen_NOT_BATCHED"
    out = Path(args.out_dir) / f"__{path.stem}__{k}k_steps_{tag}.wav"
    model.generate(mel, out, batched, target, overlap, hp.mu_law, seed=args.seed)
    print(f"wrote {out}")


if __name__ == "__main__":
    main()
