"""TTS caller on the MI355X vocoder — the WaveRNN half of the reference's gen_tacotron.py.

The reference synthesises each sentence with its PyTorch Tacotron and hands the mel to
`WaveRNN.generate()` (gen_tacotron.py:142-168):

    _, m, attention = tts_model.generate(x)          # :145
    m = (m + 4) / 8; np.clip(m, 0, 1, out=m)          # :147-148  (Tacotron scale → [0, 1])
    m = torch.tensor(m).unsqueeze(0)                  # :167
    voc_model.generate(m, save_path, batched, hp.voc_target, hp.voc_overlap, hp.mu_law)   # :168

Tacotron, the text front-end and Griffin-Lim stay outside this package (SURVEY.md §8(f)3:
"Tacotron stays PyTorch"): `synthesize()` takes any object with the reference Tacotron's
`generate(x) -> (linear, mel, attention)` and any sequence of already-encoded inputs
(`text_to_sequence` output), so the reference's own Tacotron drops in unchanged. The CLI vocodes
mels that a Tacotron run saved as .npy (Tacotron scale, before the :147 rescale):

    python -m wavernn_amd.gen_tacotron -m mel0.npy mel1.npy [-b|-u] [-t T] [-o O]
                                       [--voc_weights W.pyt] [--hp_file hparams.py]
                                       [--tts_k K] [--out_dir DIR] [--names a b ...]
"""
from __future__ import annotations

import argparse
from pathlib import Path
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

from .hparams import HParams


def tacotron_mel_to_vocoder(m) -> torch.Tensor:
    """gen_tacotron.py:147-148 and :167 — Tacotron mel (n_mels, T) in its [-4, 4] scale →
    the (1, n_mels, T) [0, 1] tensor WaveRNN.generate() expects. Same float arithmetic as the
    reference: (m + 4) / 8 in the input's dtype, then clip."""
    m = np.asarray(m)
    m = (m + 4) / 8
    np.clip(m, 0, 1, out=m)
    return torch.tensor(m).unsqueeze(0)


def output_name(i: int, v_type: str, tts_k: int, input_text: Optional[str] = None,
                standard_name: Optional[str] = None) -> str:
    """Wav file name of sentence i (1-based), gen_tacotron.py:157-162."""
    if standard_name is not None:
        return f'{standard_name}.wav'
    if input_text:
        return f'__input_{input_text[:10]}_{v_type}_{tts_k}k.wav'
    return f'{i}_{v_type}_{tts_k}k.wav'


def vocoder_type(batched: bool) -> str:
    """gen_tacotron.py:150-155 (the WaveRNN branches)."""
    return 'wavernn_batched' if batched else 'wavernn_unbatched'


def synthesize(tts_model, voc_model, inputs: Sequence, out_dir: Path, batched: bool, target: int, overlap: int,
               mu_law: bool, tts_k: int = 0, input_text: Optional[str] = None,
               standard_names: Optional[Sequence[str]] = None, seed: Optional[int] = None,
               save_attention: Optional[Callable] = None) -> List[np.ndarray]:
    """gen_tacotron.py:142-168 with the vocoder on the MI355X path: for each encoded input,
    Tacotron (PyTorch, the caller's) → rescale → `voc_model.generate()`. Returns the waveforms."""
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    v_type = vocoder_type(batched)
    wavs = []
    for i, x in enumerate(inputs, 1):
        print(f'\n| Generating {i}/{len(inputs)}')
        _, m, attention = tts_model.generate(x)
        name = output_name(i, v_type, tts_k, input_text, standard_names[i - 1] if standard_names else None)
        save_path = out_dir / name
        if save_attention is not None:
            save_attention(attention, save_path)
        mel = tacotron_mel_to_vocoder(m)
        s = None if seed is None else seed + i - 1
        wavs.append(voc_model.generate(mel, save_path, batched, target, overlap, mu_law, seed=s))
    return wavs


class _SavedMels:
    """Stands in for Tacotron when its mels were saved to disk: generate(i) → (None, mel, None)."""

    def __init__(self, paths: Sequence[Path], n_mels: int):
        self.paths = [Path(p) for p in paths]
        self.n_mels = n_mels

    def generate(self, i):
        p = self.paths[i]
        if p.suffix != '.npy':
            raise ValueError(f'Expected a .npy Tacotron mel, got {p.suffix}')
        m = np.load(p, allow_pickle=False)
        if m.ndim != 2 or m.shape[0] != self.n_mels:
            raise ValueError(f'Expected a numpy array shaped (n_mels, n_frames), but got {m.shape}!')
        return None, m, None


def main(argv=None):
    ap = argparse.ArgumentParser(description='Vocode Tacotron mels on MI355X (gen_tacotron.py, wavernn branch)')
    ap.add_argument('--mels', '-m', nargs='+', required=True, help='Tacotron mel .npy files (Tacotron scale)')
    ap.add_argument('--batched', '-b', dest='batched', action='store_true', help='Fast Batched Generation')
    ap.add_argument('--unbatched', '-u', dest='batched', action='store_false', help='Slow Unbatched Generation')
    ap.add_argument('--overlap', '-o', type=int)
    ap.add_argument('--target', '-t', type=int)
    ap.add_argument('--voc_weights', type=str, help='reference-format WaveRNN state_dict (*.pyt)')
    ap.add_argument('--hp_file', metavar='FILE', default=None)
    ap.add_argument('--tts_k', type=int, default=0, help='Tacotron step / 1000, for the file names')
    ap.add_argument('--names', nargs='*', default=None, help='output names (hp.test_sentences_names)')
    ap.add_argument('--out_dir', default='.')
    ap.add_argument('--seed', type=int, default=None)
    ap.set_defaults(batched=None)
    args = ap.parse_args(argv)
    hp = HParams().configure(args.hp_file)
    target = args.target if args.target is not None else hp.voc_target
    overlap = args.overlap if args.overlap is not None else hp.voc_overlap
    batched = args.batched if args.batched is not None else hp.voc_gen_batched
    if args.names is not None and len(args.names) != len(args.mels):
        raise ValueError('--names needs one name per mel')
    if not torch.cuda.is_available():
        raise RuntimeError('the MI355X generation path needs a GPU')
    from .gen_wavernn import build_model
    voc = build_model(hp, torch.device('cuda'))
    if args.voc_weights:
        voc.load(args.voc_weights)
    tts = _SavedMels(args.mels, hp.num_mels)
    synthesize(tts, voc, list(range(len(args.mels))), Path(args.out_dir), batched, target, overlap, hp.mu_law,
               tts_k=args.tts_k, standard_names=args.names, seed=args.seed)
    print('\n\nDone.\n')


if __name__ == '__main__':
    main()
