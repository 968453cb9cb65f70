"""Drop-in `WaveRNN` for models/fatchord_version.py whose generate() runs on MI355X.

Same constructor, submodule names, state_dict keys (so `load()` takes the reference's
`*.pyt` checkpoints), `get_step`, `load`, `save` and `generate(mels, save_path, batched,
target, overlap, mu_law)` contract as the reference (fatchord_version.py:92-435).  What
changes is where the sample loop runs: instead of the host-driven per-step loop
(:201-241), generate() packs the upsampled conditioning time-major and calls ONE persistent
HIP kernel through the C-ABI (`FatchordLoop`).  There is no CPU fallback: the model must
live on a GPU and the HIP library must be built, otherwise generate() raises.

Pre-processing: MelResNet as ONE fused HIP kernel (`wrnn_melresnet`, every BatchNorm folded on the
host; the torch module only for channel counts the kernel does not cover), then the loop entry
`wrnn_generate_frames`: pad + the stretch/box-conv chain + crop + aux stretch + fold are applied to
the conditioning TERMS at frame rate on the XCD-resident paths (csrc/frame_terms.hip), or through
the per-sample records of `condition.upsample_pack` on the others.
Post-processing (mu-law, cross-fade/unfold, trim, fade-out) is one float64 HIP kernel
(`condition.postprocess`) with the reference's operation order; only the finished waveform
crosses to the host.
"""
from __future__ import annotations

import os
import time
from pathlib import Path
from typing import List, Optional, Sequence, Union

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as nat
from . import condition, dsp
from .loop import LOOP_KEYS, FatchordLoop, noise_width


# --------------------------------------------------------------------- upsample network
class ResBlock(nn.Module):
    """1×1 conv → BN → ReLU → 1×1 conv → BN, plus identity (fatchord_version.py:13-28)."""

    def __init__(self, dims):
        super().__init__()
        self.conv1 = nn.Conv1d(dims, dims, kernel_size=1, bias=False)
        self.conv2 = nn.Conv1d(dims, dims, kernel_size=1, bias=False)
        self.batch_norm1 = nn.BatchNorm1d(dims)
        self.batch_norm2 = nn.BatchNorm1d(dims)

    def forward(self, x):
        y = F.relu(self.batch_norm1(self.conv1(x)))
        return self.batch_norm2(self.conv2(y)) + x


class MelResNet(nn.Module):
    """Valid conv (k = 2·pad+1) → BN → ReLU → res blocks → 1×1 conv (fatchord_version.py:31-48)."""

    def __init__(self, res_blocks, in_dims, compute_dims, res_out_dims, pad):
        super().__init__()
        self.conv_in = nn.Conv1d(in_dims, compute_dims, kernel_size=2 * pad + 1, bias=False)
        self.batch_norm = nn.BatchNorm1d(compute_dims)
        self.layers = nn.ModuleList([ResBlock(compute_dims) for _ in range(res_blocks)])
        self.conv_out = nn.Conv1d(compute_dims, res_out_dims, kernel_size=1)

    def forward(self, x):
        x = F.relu(self.batch_norm(self.conv_in(x)))
        for layer in self.layers:
            x = layer(x)
        return self.conv_out(x)


class Stretch2d(nn.Module):
    """Nearest-neighbour repeat along (freq, time) (fatchord_version.py:51-61)."""

    def __init__(self, x_scale, y_scale):
        super().__init__()
        self.x_scale, self.y_scale = x_scale, y_scale

    def forward(self, x):
        return x.repeat_interleave(self.y_scale, dim=2).repeat_interleave(self.x_scale, dim=3)


class UpsampleNetwork(nn.Module):
    """MelResNet aux features stretched ×hop, and the mel upsampled by per-factor
    stretch + (1, 2s+1) box convs, cropped by pad·hop each side (fatchord_version.py:64-89).
    Returns (mels [B][L][feat], aux [B][L][res_out]) as contiguous time-major tensors."""

    def __init__(self, feat_dims, upsample_scales, compute_dims, res_blocks, res_out_dims, pad):
        super().__init__()
        total_scale = int(np.prod(upsample_scales))
        self.indent = pad * total_scale
        self.resnet = MelResNet(res_blocks, feat_dims, compute_dims, res_out_dims, pad)
        self.resnet_stretch = Stretch2d(total_scale, 1)
        self.up_layers = nn.ModuleList()
        for scale in upsample_scales:
            k = 2 * scale + 1
            conv = nn.Conv2d(1, 1, kernel_size=(1, k), padding=(0, scale), bias=False)
            conv.weight.data.fill_(1.0 / k)
            self.up_layers.append(Stretch2d(scale, 1))
            self.up_layers.append(conv)

    def forward(self, m):
        aux = self.resnet_stretch(self.resnet(m).unsqueeze(1)).squeeze(1)
        m = m.unsqueeze(1)
        for f in self.up_layers:
            m = f(m)
        m = m.squeeze(1)[:, :, self.indent:-self.indent]
        return m.transpose(1, 2), aux.transpose(1, 2)


# ------------------------------------------------------------------------------ model
class WaveRNN(nn.Module):
    def __init__(self, rnn_dims, fc_dims, bits, pad, upsample_factors, feat_dims, compute_dims,
                 res_out_dims, res_blocks, hop_length, sample_rate, mode='RAW'):
        super().__init__()
        self.mode = mode
        self.pad = pad
        if mode == 'RAW':
            self.n_classes = 2 ** bits
        elif mode == 'MOL':
            self.n_classes = 30
        else:
            raise RuntimeError("Unknown model mode value - ", mode)
        self.rnn_dims = rnn_dims
        self.fc_dims = fc_dims
        self.feat_dims = feat_dims
        self.aux_dims = res_out_dims // 4
        self.hop_length = hop_length
        self.sample_rate = sample_rate
        self.upsample = UpsampleNetwork(feat_dims, upsample_factors, compute_dims, res_blocks, res_out_dims, pad)
        self.I = nn.Linear(feat_dims + self.aux_dims + 1, rnn_dims)
        self.rnn1 = nn.GRU(rnn_dims, rnn_dims, batch_first=True)
        self.rnn2 = nn.GRU(rnn_dims + self.aux_dims, rnn_dims, batch_first=True)
        self.fc1 = nn.Linear(rnn_dims + self.aux_dims, fc_dims)
        self.fc2 = nn.Linear(fc_dims + self.aux_dims, fc_dims)
        self.fc3 = nn.Linear(fc_dims, self.n_classes)
        self.register_buffer('step', torch.zeros(1, dtype=torch.long))
        self.num_params()
        self._loop: Optional[FatchordLoop] = None
        self._loop_key = None
        self.last_gen_seconds = 0.0

    # -------------------------------------------------------------- training forward
    def forward(self, x, mels):
        """Teacher-forced forward (fatchord_version.py:131-167); training is out of scope for
        the MI355X path, this keeps the module usable with the reference's train loop."""
        self.step += 1
        b = x.size(0)
        h1 = torch.zeros(1, b, self.rnn_dims, device=x.device)
        h2 = torch.zeros(1, b, self.rnn_dims, device=x.device)
        mels, aux = self.upsample(mels)
        a1, a2, a3, a4 = aux.split(self.aux_dims, dim=2)
        x = self.I(torch.cat([x.unsqueeze(-1), mels, a1], dim=2))
        res = x
        x, _ = self.rnn1(x, h1)
        x = x + res
        res = x
        x, _ = self.rnn2(torch.cat([x, a2], dim=2), h2)
        x = x + res
        x = F.relu(self.fc1(torch.cat([x, a3], dim=2)))
        x = F.relu(self.fc2(torch.cat([x, a4], dim=2)))
        return self.fc3(x)

    # -------------------------------------------------------------------- loop handle
    def _loop_params(self):
        sd = dict(self.named_parameters())
        return {k: sd[k] for k in LOOP_KEYS}

    def loop_handle(self, grid: int = 0) -> FatchordLoop:
        """The device handle, (re)packed whenever the loop weights changed (load, training)."""
        device = next(self.parameters()).device
        if device.type != 'cuda':
            raise RuntimeError("WaveRNN.generate runs on the MI355X HIP path: move the model to a GPU "
                               "(model.to('cuda')); there is no CPU fallback")
        params = self._loop_params()
        key = (device.index or 0, grid) + tuple((p.data_ptr(), p._version) for p in params.values())
        if self._loop is None or self._loop_key is None or self._loop_key[:2] != key[:2]:
            if self._loop is not None:
                self._loop.close()
            self._loop = FatchordLoop(self.mode, self.rnn_dims, self.fc_dims, self.aux_dims, self.feat_dims,
                                      self.n_classes, device=device.index or 0, grid=grid)
            self._loop_key = None
        if self._loop_key != key:
            self._loop.set_weights(params)
            self._loop_key = key
        return self._loop

    # ---------------------------------------------------------------------- generate
    def _upsample_spec(self) -> condition.UpsampleSpec:
        """Host copy of the box-conv taps, refreshed when those parameters change."""
        convs = [m.weight for m in self.upsample.up_layers if isinstance(m, nn.Conv2d)]
        key = tuple((w.data_ptr(), w._version) for w in convs)
        if getattr(self, "_up_key", None) != key:
            self._up_spec = condition.UpsampleSpec.from_module(self.upsample, self.feat_dims, self.pad)
            self._up_key = key
        return self._up_spec

    @torch.no_grad()
    def frames(self, mels):
        """generate()'s inputs at frame rate: (mel [U][feat][T], MelResNet(pad_tensor(mel))
        [U][res_out][T], wave_len) — fatchord_version.py:183-186 up to the upsampling, which the
        loop entry (wrnn_generate_frames) or condition.upsample_pack performs on the device."""
        device = next(self.parameters()).device
        if device.type != 'cuda':
            raise RuntimeError("WaveRNN.generate runs on the MI355X HIP path: move the model to a GPU "
                               "(model.to('cuda')); there is no CPU fallback")
        was_training = self.training
        self.eval()
        try:
            mels = torch.as_tensor(mels, device=device).to(torch.float32)
            wave_len = (mels.size(-1) - 1) * self.hop_length
            padded = self.pad_tensor(mels.transpose(1, 2), pad=self.pad, side='both').transpose(1, 2)
            aux = self._melresnet(padded)
        finally:
            self.train(was_training)
        return mels.contiguous(), aux.contiguous().float(), wave_len

    def _melresnet(self, padded):
        """MelResNet(padded) through the fused HIP kernel (wrnn_melresnet: every BatchNorm folded,
        one launch); the torch module (MIOpen) only for channel counts the kernel does not cover."""
        res = self.upsample.resnet
        if os.environ.get("WRNN_TORCH_MELRESNET"):   # A/B: the torch module (MIOpen)
            return res(padded)
        key = tuple((p.data_ptr(), p._version) for p in res.parameters()) + \
            tuple((b.data_ptr(), b._version) for b in res.buffers())
        if getattr(self, "_mr_key", None) != key:
            self._mr_cfg = condition.melresnet_cfg(res)
            self._mr_packed = condition.melresnet_pack(res)
            self._mr_key = key
        try:
            return condition.melresnet(self._mr_cfg, self._mr_packed, padded)
        except nat.WrnnError as e:
            if e.code != -6:   # WRNN_EUNSUPPORTED
                raise
            return res(padded)

    @torch.no_grad()
    def conditioning(self, mels, batched, target, overlap):
        """pad → upsample → (fold) → time-major [L][B][feat + 4·aux] (fatchord_version.py:183-190).
        MelResNet in eval form (BatchNorm running statistics, folded) is the `wrnn_melresnet` HIP
        kernel; everything after it the `wrnn_upsample_pack` HIP kernel."""
        mels, aux, wave_len = self.frames(mels)
        cond = condition.upsample_pack(self._upsample_spec(), mels, aux, target if batched else 0, overlap)
        return cond, wave_len

    def generate(self, mels, save_path: Union[str, Path, None], batched, target, overlap, mu_law, *,
                 noise=None, seed: Optional[int] = None, row_offset: int = 0, verbose: bool = True):
        """fatchord_version.py:169-264 with the loop on the GPU.

        Keyword-only extensions: `noise` [L][B][K] injects the sampler draws in reference order
        (parity testing); otherwise draws come from in-kernel Philox keyed by `seed` (default:
        drawn from torch's global RNG, so torch.manual_seed governs reproducibility) and by the
        global row id `row_offset + b` of each loop row b (a fold when batched) — the key that
        makes `generate_many` and the sharded entry points reproduce single calls."""
        self.eval()
        mu_law = mu_law if self.mode == 'RAW' else False
        start = time.time()
        with torch.no_grad():
            # the loop takes the frames: pad → upsample → fold happen inside wrnn_generate_frames
            # (the conditioning terms formed at frame rate, csrc/frame_terms.hip)
            mel_f, aux, wave_len = self.frames(mels)
            loop = self.loop_handle()
            nz = None
            if noise is not None:
                nz = torch.as_tensor(noise, dtype=torch.float32).to(mel_f.device).contiguous()
            if seed is None:
                seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            out, _ = loop.generate_frames(self._upsample_spec(), mel_f, aux, target if batched else 0, overlap,
                                          noise=nz, seed=seed, row_offset=row_offset)
            b_size, seq_len = out.shape
            # mu-law, xfade_and_unfold / row 0, trim, fade-out (:243-258) in float64 on the device
            output = condition.postprocess(out, batched, overlap, mu_law, self.n_classes, wave_len,
                                           20 * self.hop_length).cpu().numpy()
        self.last_gen_seconds = time.time() - start
        if verbose:
            self.gen_display(seq_len - 1, seq_len, b_size, start)
        dsp.save_wav(output, save_path, self.sample_rate)
        self.train()
        return output

    def rows_of(self, n_frames: int, batched: bool, target: int, overlap: int) -> int:
        """Loop rows generate() runs for a mel of n_frames frames: 1, or its fold count."""
        if not batched:
            return 1
        return self.fold_count(n_frames * self.hop_length, target, overlap)[0]

    def _mel_list(self, mels: Sequence) -> List[torch.Tensor]:
        device = next(self.parameters()).device
        ms = [torch.as_tensor(m, device=device).to(torch.float32) for m in mels]
        ms = [m if m.dim() == 3 else m[None] for m in ms]
        if not ms or any(m.dim() != 3 or m.shape[0] != 1 or m.shape[1] != self.feat_dims for m in ms):
            raise ValueError(f"mels must be a non-empty sequence of (1, {self.feat_dims}, T) arrays")
        return ms

    @torch.no_grad()
    def conditioning_many(self, mels: Sequence, batched: bool, target: int, overlap: int):
        """Conditioning of several utterances as the rows of ONE loop launch.

        Returns (cond [L][rows][C], per-utterance (first row, rows, steps, wave_len)).  Unbatched:
        row i is utterance i, its records padded with zeros after its own L_i steps (a row's
        samples depend only on earlier steps, so trimming to L_i is exact).  Batched: the folds
        of utterance i are rows [r_i, r_i + nf_i), all folds sharing the window target + 2·overlap.
        Mels of one length go through MelResNet and the upsample kernel together."""
        ms = self._mel_list(mels)
        device = ms[0].device
        if len({m.shape[2] for m in ms}) == 1:
            cond, wave_len = self.conditioning(torch.cat(ms, 0), batched, target, overlap)
            per = cond.shape[1] // len(ms)
            return cond, [(i * per, per, cond.shape[0], wave_len) for i in range(len(ms))]
        parts = [self.conditioning(m, batched, target, overlap) for m in ms]
        L = max(c.shape[0] for c, _ in parts)
        rows = sum(c.shape[1] for c, _ in parts)
        cond = torch.zeros(L, rows, parts[0][0].shape[2], dtype=torch.float32, device=device)
        spans, r = [], 0
        for c, wave_len in parts:
            cond[:c.shape[0], r:r + c.shape[1]] = c
            spans.append((r, c.shape[1], c.shape[0], wave_len))
            r += c.shape[1]
        return cond, spans

    def generate_many(self, mels: Sequence, save_paths: Optional[Sequence] = None, batched: bool = False,
                      target: int = 11000, overlap: int = 550, mu_law: bool = True, *, noise=None,
                      seed: Optional[int] = None, row_offset: int = 0, verbose: bool = False) -> List[np.ndarray]:
        """generate() for several utterances in ONE persistent-kernel launch (the utterances —
        or, batched, all their folds — are the launch's rows).  The reference vocodes a list one
        generate() at a time (gen_wavernn.py:11-35, gen_tacotron.py:142-168); this returns the
        same list of float64 waveforms.  Utterance i's rows are keyed row_offset + (rows of the
        utterances before it) + j, so under Philox `generate_many(mels, seed=s)[i]` equals
        `generate(mels[i], seed=s, row_offset=<that first row>)` bit for bit.  `noise`, when given,
        is [L_max][rows][K] in that row order."""
        self.eval()
        mu_law = mu_law if self.mode == 'RAW' else False
        start = time.time()
        with torch.no_grad():
            ms = self._mel_list(mels)
            loop = self.loop_handle()
            if seed is None:
                seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            dev = next(self.parameters()).device
            nz = None if noise is None else torch.as_tensor(noise, dtype=torch.float32).to(dev).contiguous()
            if len({m.shape[2] for m in ms}) == 1:
                # one length: the frames of all utterances go to the loop entry together
                mel_f, aux, wave_len = self.frames(torch.cat(ms, 0))
                out, _ = loop.generate_frames(self._upsample_spec(), mel_f, aux, target if batched else 0, overlap,
                                              noise=nz, seed=seed, row_offset=row_offset)
                per = out.shape[0] // len(ms)
                spans = [(i * per, per, out.shape[1], wave_len) for i in range(len(ms))]
            else:
                cond, spans = self.conditioning_many(ms, batched, target, overlap)
                out, _ = loop.generate(cond, noise=nz, seed=seed, row_offset=row_offset)
            waves = [condition.postprocess(out[r0:r0 + n, :steps], batched, overlap, mu_law, self.n_classes,
                                           wave_len, 20 * self.hop_length)
                     for r0, n, steps, wave_len in spans]
            outputs = [w.cpu().numpy() for w in waves]
        self.last_gen_seconds = time.time() - start
        if verbose:
            self.gen_display(out.shape[1] - 1, out.shape[1], out.shape[0], start)
        for i, output in enumerate(outputs):
            if save_paths is not None and save_paths[i] is not None:
                dsp.save_wav(output, save_paths[i], self.sample_rate)
        self.train()
        return outputs

    def gen_display(self, i, seq_len, b_size, start):
        gen_rate = (i + 1) / max(time.time() - start, 1e-9) * b_size / 1000
        print(f'| {i + 1}/{seq_len} steps × {b_size} rows | Gen Rate: {gen_rate:.1f}kHz |')

    def get_gru_cell(self, gru):
        """nn.GRUCell view of a single-layer GRU's weights (fatchord_version.py:273-279)."""
        cell = nn.GRUCell(gru.input_size, gru.hidden_size).to(gru.weight_hh_l0.device)
        cell.weight_hh.data = gru.weight_hh_l0.data
        cell.weight_ih.data = gru.weight_ih_l0.data
        cell.bias_hh.data = gru.bias_hh_l0.data
        cell.bias_ih.data = gru.bias_ih_l0.data
        return cell

    @staticmethod
    def pad_tensor(x, pad, side='both'):
        """Zero-pad the time axis of [b][t][c] (fatchord_version.py:281-291)."""
        b, t, c = x.size()
        total = t + 2 * pad if side == 'both' else t + pad
        padded = torch.zeros(b, total, c, device=x.device, dtype=x.dtype)
        if side in ('before', 'both'):
            padded[:, pad:pad + t, :] = x
        elif side == 'after':
            padded[:, :t, :] = x
        return padded

    @staticmethod
    def fold_count(total_len, target, overlap):
        n = (total_len - overlap) // (target + overlap)
        remaining = total_len - (n * (overlap + target) + overlap)
        return n + (1 if remaining != 0 else 0), remaining

    def fold_with_overlap(self, x, target, overlap):
        """[1][L][F] → [num_folds][target + 2·overlap][F]; consecutive folds share `overlap`
        steps, the tail is zero-padded (fatchord_version.py:293-340)."""
        _, total_len, features = x.size()
        num_folds, remaining = self.fold_count(total_len, target, overlap)
        if remaining != 0:
            x = self.pad_tensor(x, target + 2 * overlap - remaining, side='after')
        win = target + 2 * overlap
        folds = x[0].unfold(0, win, target + overlap)          # [n][F][win] views
        return folds[:num_folds].transpose(1, 2).contiguous()

    @staticmethod
    def xfade_and_unfold(y, target, overlap):
        """Equal-power cross-fade of folds and overlap-add back to 1-D float64
        (fatchord_version.py:342-405; `fade_out` keeps the reference's leading ones).  Host
        numpy for callers of the reference API; generate() runs the device kernel
        (`condition.postprocess`)."""
        num_folds, length = y.shape
        target = length - 2 * overlap
        total_len = num_folds * (target + overlap) + overlap
        silence_len = overlap // 2
        fade_len = overlap - silence_len
        t = np.linspace(-1, 1, fade_len, dtype=np.float64)
        fade_in = np.concatenate([np.zeros(silence_len, dtype=np.float64), np.sqrt(0.5 * (1 + t))])
        fade_out = np.concatenate([np.ones(silence_len, dtype=np.float64), np.sqrt(0.5 * (1 - t))])
        y = np.array(y, dtype=np.float64, copy=True)
        y[:, :overlap] *= fade_in
        y[:, -overlap:] *= fade_out
        unfolded = np.zeros(total_len, dtype=np.float64)
        for i in range(num_folds):
            s = i * (target + overlap)
            unfolded[s:s + length] += y[i]
        return unfolded

    # ------------------------------------------------------------------ bookkeeping
    def get_step(self):
        return self.step.data.item()

    def log(self, path, msg):
        with open(path, 'a') as f:
            print(msg, file=f)

    def load(self, path: Union[str, Path]):
        """Reference checkpoint (a state_dict saved with torch.save) → this model.  Loaded
        with weights_only=True: a checkpoint never executes code."""
        device = next(self.parameters()).device
        self.load_state_dict(torch.load(path, map_location=device, weights_only=True), strict=False)

    def save(self, path: Union[str, Path]):
        torch.save(self.state_dict(), path)

    def num_params(self, print_out=True):
        n = sum(p.numel() for p in self.parameters() if p.requires_grad) / 1_000_000
        if print_out:
            print('Trainable Parameters: %.3fM' % n)
        return n

    def noise_width(self) -> int:
        return noise_width(self.mode, self.n_classes)
