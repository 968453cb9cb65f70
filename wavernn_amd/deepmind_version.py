"""Drop-in for the reference `models.deepmind_version.WaveRNN` (dual coarse/fine 8-bit softmax,
BASELINE config 5) whose `generate()` runs on the MI355X persistent kernels instead of the
per-step eager loop (:98-156): wavernn_amd/csrc/deepmind_xcd.hip for hidden 896 / quantisation
256 (4 rows per XCD, 32 per launch), deepmind_rows.hip for other sizes.

Same constructor (hidden_size, quantisation), parameter names (so `load_state_dict` takes the
reference's state_dicts), training `forward` (:37-72) and `generate(seq_len)` return contract
`(output, coarse, fine)` (:158-163; output = coarse·256 + fine − 2^15, utils/dsp.py:33-34).
Keyword-only extensions: `batch` (independent rows in one launch), `noise` (inject the
Categorical draws, [L][batch][2·quantisation] Exp(1): coarse q then fine q per step), `seed`
(in-kernel Philox).  There is no CPU fallback: a CPU model raises.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .loop import DM_KEYS, DeepmindLoop


class WaveRNN(nn.Module):
    def __init__(self, hidden_size=896, quantisation=256):
        super().__init__()
        self.hidden_size = hidden_size
        self.split_size = hidden_size // 2
        # the main matmul (deepmind_version.py:16) and output / input layers (:19-26)
        self.R = nn.Linear(self.hidden_size, 3 * self.hidden_size, bias=False)
        self.O1 = nn.Linear(self.split_size, self.split_size)
        self.O2 = nn.Linear(self.split_size, quantisation)
        self.O3 = nn.Linear(self.split_size, self.split_size)
        self.O4 = nn.Linear(self.split_size, quantisation)
        self.I_coarse = nn.Linear(2, 3 * self.split_size, bias=False)
        self.I_fine = nn.Linear(3, 3 * self.split_size, bias=False)
        # gate biases (:29-31)
        self.bias_u = nn.Parameter(torch.zeros(self.hidden_size))
        self.bias_r = nn.Parameter(torch.zeros(self.hidden_size))
        self.bias_e = nn.Parameter(torch.zeros(self.hidden_size))
        self.quantisation = quantisation
        self._loop: Optional[DeepmindLoop] = None
        self._loop_key = None
        self.num_params()

    def forward(self, prev_y, prev_hidden, current_coarse):
        """Teacher-forced step for training (deepmind_version.py:37-72)."""
        R_hidden = self.R(prev_hidden)
        R_u, R_r, R_e = torch.split(R_hidden, self.hidden_size, dim=1)
        I_coarse_u, I_coarse_r, I_coarse_e = torch.split(self.I_coarse(prev_y), self.split_size, dim=1)
        fine_input = torch.cat([prev_y, current_coarse], dim=1)
        I_fine_u, I_fine_r, I_fine_e = torch.split(self.I_fine(fine_input), self.split_size, dim=1)
        I_u = torch.cat([I_coarse_u, I_fine_u], dim=1)
        I_r = torch.cat([I_coarse_r, I_fine_r], dim=1)
        I_e = torch.cat([I_coarse_e, I_fine_e], dim=1)
        u = torch.sigmoid(R_u + I_u + self.bias_u)
        r = torch.sigmoid(R_r + I_r + self.bias_r)
        e = torch.tanh(r * R_e + I_e + self.bias_e)
        hidden = u * prev_hidden + (1. - u) * e
        hidden_coarse, hidden_fine = torch.split(hidden, self.split_size, dim=1)
        out_coarse = self.O2(F.relu(self.O1(hidden_coarse)))
        out_fine = self.O4(F.relu(self.O3(hidden_fine)))
        return out_coarse, out_fine, hidden

    def _loop_params(self):
        sd = dict(self.named_parameters())
        return {k: sd[k] for k in DM_KEYS}

    def loop_handle(self, grid: int = 0) -> DeepmindLoop:
        """The device handle, (re)packed whenever the weights changed (load, training)."""
        device = next(self.parameters()).device
        if device.type != 'cuda':
            raise RuntimeError("WaveRNN.generate runs on the MI355X HIP path: move the model to a GPU "
                               "(model.to('cuda')); there is no CPU fallback")
        params = self._loop_params()
        key = (device.index or 0, grid) + tuple((p.data_ptr(), p._version) for p in params.values())
        if self._loop is None or self._loop_key is None or self._loop_key[:2] != key[:2]:
            if self._loop is not None:
                self._loop.close()
            self._loop = DeepmindLoop(self.hidden_size, self.quantisation, device=device.index or 0, grid=grid)
            self._loop_key = None
        if self._loop_key != key:
            self._loop.set_weights(params)
            self._loop_key = key
        return self._loop

    @torch.no_grad()
    def generate(self, seq_len, *, batch: int = 1, noise=None, seed: Optional[int] = None, row_offset: int = 0):
        """deepmind_version.py:75-165.  Returns (output, coarse, fine) as numpy int64 arrays of
        shape (seq_len,) for batch = 1 (the reference contract), (batch, seq_len) otherwise.
        Row b's Philox draws are keyed (seed, row_offset + b): a row generated alone with its
        row_offset equals the same row of a batch (the sharded entry point relies on it)."""
        loop = self.loop_handle()
        device = next(self.parameters()).device
        if noise is not None:
            noise = torch.as_tensor(np.asarray(noise, dtype=np.float32)).to(device).contiguous()
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        _, comb = loop.generate(batch, seq_len, noise=noise, seed=seed, row_offset=row_offset, device=device)
        output = comb.cpu().numpy().astype(np.int64)
        unsigned = output + 2 ** 15                      # split_signal, utils/dsp.py:25-29
        coarse, fine = unsigned // 256, unsigned % 256
        if batch == 1:
            return output[0], coarse[0], fine[0]
        return output, coarse, fine

    def get_initial_hidden(self, batch_size=1):
        device = next(self.parameters()).device
        return torch.zeros(batch_size, self.hidden_size, device=device)

    def num_params(self, print_out=True):
        n = sum(p.numel() for p in self.parameters() if p.requires_grad) / 1_000_000
        if print_out:
            print('Trainable Parameters: %.3f million' % n)
        return n
