"""PyTorch-CPU eager restatement of the reference generate() — bench.py's `cpu_baseline`.

TEST / BENCH INFRASTRUCTURE ONLY (like the rest of oracle/): imported by bench.py's cpu_baseline
leg and by tests, never by the product package.

SURVEY.md §8(d) asks for the reference's own op sequence timed on the GPU box's host cores, and
the reference Python does not travel.  This is that op sequence, written from the reference's
behaviour with the same eager torch ops on the CPU:

  pad + UpsampleNetwork   fatchord_version.py:183-186, :13-89 (conv1d / batch_norm / relu,
                          nearest stretch = repeat_interleave, Conv2d (1, 2s+1) box filters, crop)
  fold_with_overlap       :188-190 (oracle.py's numpy version: a copy, not arithmetic)
  sample loop             :192-241 — per step: cat, I (linear), gru_cell, residual, gru_cell,
                          residual, cat + fc1 + relu, cat + fc2 + relu, fc3, then the MoL sampler
                          (utils/distribution.py:87-123) or softmax + Categorical (:231-237)
  post                    :243-258 (float64 numpy, oracle.postprocess)
  deepmind loop           models/deepmind_version.py:98-156 (config 5's cpu_baseline): R, the
                          coarse gates, O1/O2 + softmax + Categorical, the fine half likewise

The sampler draws are injected ([L][B][K], the reference draw order of SURVEY.md §8(b)), so
the result can be checked against the C oracle (tests/test_torch_cpu_baseline.py)."""
from __future__ import annotations

import time
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import oracle

LN_1E14 = -32.23619130191664   # log(1e-14): the log-scale floor of distribution.py:114-115


def _t(state, k):
    return torch.as_tensor(np.asarray(state[k]), dtype=torch.float32)


def upsample(state, dims, mel: torch.Tensor):
    """mel [1][feat][T] → (mels [1][L][feat], aux [1][L][4·aux]) on the CPU (fatchord_version.py:82-89)."""
    p = "upsample.resnet."
    x = F.pad(mel, (dims.pad, dims.pad))                                          # pad_tensor (:185, :281-291)
    y = F.conv1d(x, _t(state, p + "conv_in.weight"))                               # MelResNet (:31-48)

    def bn(v, q):
        return F.batch_norm(v, _t(state, q + ".running_mean"), _t(state, q + ".running_var"),
                            _t(state, q + ".weight"), _t(state, q + ".bias"), False, 0.0, 1e-5)

    y = F.relu(bn(y, p + "batch_norm"))
    for i in range(dims.res_blocks):                                               # ResBlock (:13-28)
        q = p + f"layers.{i}"
        r = y
        y = F.relu(bn(F.conv1d(y, _t(state, q + ".conv1.weight")), q + ".batch_norm1"))
        y = bn(F.conv1d(y, _t(state, q + ".conv2.weight")), q + ".batch_norm2") + r
    aux = F.conv1d(y, _t(state, p + "conv_out.weight"), _t(state, p + "conv_out.bias"))
    total = int(np.prod(dims.upsample_factors))
    aux = aux.repeat_interleave(total, dim=2)                                      # resnet_stretch (:83)
    m = x.unsqueeze(1)                                                             # [1][1][feat][T+2pad]
    for i, s in enumerate(dims.upsample_factors):
        m = m.repeat_interleave(s, dim=3)                                          # Stretch2d(s, 1)
        m = F.conv2d(m, _t(state, f"upsample.up_layers.{2 * i + 1}.weight"), padding=(0, s))
    indent = dims.pad * total
    m = m.squeeze(1)[:, :, indent:-indent]                                         # (:88)
    return m.transpose(1, 2).contiguous(), aux.transpose(1, 2).contiguous()


def loop(state: Dict[str, np.ndarray], mode: str, mels: torch.Tensor, aux: torch.Tensor, noise: np.ndarray,
         steps: Optional[int] = None) -> np.ndarray:
    """The per-step loop (fatchord_version.py:192-241) on [B][L][feat] / [B][L][4·A] conditioning
    for `steps` steps (default all); noise [L][B][K].  Returns samples [B][steps] (float32)."""
    B, L, _ = mels.shape
    steps = L if steps is None else min(steps, L)
    A = aux.shape[2] // 4
    I_w, I_b = _t(state, "I.weight"), _t(state, "I.bias")
    g1 = [_t(state, "rnn1." + k) for k in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0")]
    g2 = [_t(state, "rnn2." + k) for k in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0")]
    W1, b1, W2, b2 = _t(state, "fc1.weight"), _t(state, "fc1.bias"), _t(state, "fc2.weight"), _t(state, "fc2.bias")
    W3, b3 = _t(state, "fc3.weight"), _t(state, "fc3.bias")
    R, nc = I_w.shape[0], W3.shape[0]
    nz = torch.as_tensor(np.ascontiguousarray(noise[:steps]), dtype=torch.float32)
    out = torch.empty(B, steps)
    x = torch.zeros(B, 1)
    h1 = torch.zeros(B, R)
    h2 = torch.zeros(B, R)
    with torch.no_grad():
        for i in range(steps):
            m_t = mels[:, i, :]                                                      # (:203-206)
            a1, a2, a3, a4 = (aux[:, i, A * j:A * (j + 1)] for j in range(4))
            x = F.linear(torch.cat([x, m_t, a1], dim=1), I_w, I_b)                  # (:208-209)
            h1 = torch.gru_cell(x, h1, *g1)                                          # (:210)
            x = x + h1                                                               # (:212)
            h2 = torch.gru_cell(torch.cat([x, a2], dim=1), h2, *g2)                  # (:213-214)
            x = x + h2                                                               # (:216)
            x = F.relu(F.linear(torch.cat([x, a3], dim=1), W1, b1))                  # (:217-218)
            x = F.relu(F.linear(torch.cat([x, a4], dim=1), W2, b2))                  # (:220-221)
            logits = F.linear(x, W3, b3)                                             # (:223)
            if mode == "MOL":                                                        # distribution.py:87-123
                u1, u2 = nz[i, :, :10], nz[i, :, 10]
                sel = (logits[:, :10] - torch.log(-torch.log(u1))).argmax(dim=1)
                oh = F.one_hot(sel, 10).to(torch.float32)
                mean = (logits[:, 10:20] * oh).sum(dim=1)
                log_s = torch.clamp((logits[:, 20:30] * oh).sum(dim=1), min=LN_1E14)
                s = mean + torch.exp(log_s) * (torch.log(u2) - torch.log(1.0 - u2))
                s = torch.clamp(s, -1.0, 1.0)
            else:                                                                    # (:231-237)
                probs = F.softmax(logits, dim=1)
                label = (probs / nz[i]).argmax(dim=1)                                # Categorical.sample
                s = 2.0 * label.to(torch.float32) / (nc - 1.0) - 1.0
            out[:, i] = s
            x = s.unsqueeze(1)                                                       # (:229, :237)
    return out.numpy()


def timed_generate(state, dims, mel: np.ndarray, batched: bool, target: int, overlap: int, mu_law: bool,
                   noise: np.ndarray, loop_steps: Optional[int] = None, threads: Optional[int] = None) -> dict:
    """generate() on the CPU with per-phase wall times; the loop runs `loop_steps` of its L steps
    (a bounded sample), pre- and post-processing run in full.  Returns the timings, the loop
    output and L."""
    if threads:
        torch.set_num_threads(threads)
    t0 = time.perf_counter()
    with torch.no_grad():
        m, a = upsample(state, dims, torch.as_tensor(mel, dtype=torch.float32)[None])
    if batched:                                                                      # (:188-190)
        m = torch.from_numpy(oracle.fold_with_overlap(m.numpy(), target, overlap))
        a = torch.from_numpy(oracle.fold_with_overlap(a.numpy(), target, overlap))
    t1 = time.perf_counter()
    B, L, _ = m.shape
    n = L if loop_steps is None else min(loop_steps, L)
    out = loop(state, dims.mode, m, a, noise, n)
    t2 = time.perf_counter()
    full = np.zeros((B, L), np.float32)
    full[:, :n] = out
    T = mel.shape[-1]
    wave = oracle.postprocess(full, batched, overlap, mu_law if dims.mode == "RAW" else False, dims.n_classes,
                              (T - 1) * dims.hop_length, 20 * dims.hop_length)
    t3 = time.perf_counter()
    return {"pre_s": t1 - t0, "loop_s": t2 - t1, "post_s": t3 - t2, "loop_steps": n, "L": L, "rows": B,
            "out": out, "wave": wave, "threads": torch.get_num_threads()}


def deepmind_loop(state: Dict[str, np.ndarray], B: int, noise: np.ndarray, steps: int) -> np.ndarray:
    """deepmind_version.py:98-156 for B independent rows (the reference runs one), `steps` steps;
    noise [L][B][2Q] Exp(1) (coarse q, then fine q; Categorical.sample ≡ argmax(probs / q)).
    Returns output [B][steps] int64 = coarse·256 + fine − 2^15 (utils/dsp.py:33-34)."""
    R = _t(state, "R.weight")
    O1w, O1b, O2w, O2b = (_t(state, k) for k in ("O1.weight", "O1.bias", "O2.weight", "O2.bias"))
    O3w, O3b, O4w, O4b = (_t(state, k) for k in ("O3.weight", "O3.bias", "O4.weight", "O4.bias"))
    Ic, If = _t(state, "I_coarse.weight"), _t(state, "I_fine.weight")
    H = R.shape[1]
    S, Q = H // 2, O2w.shape[0]
    bu, br, be = (_t(state, k) for k in ("bias_u", "bias_r", "bias_e"))
    (bcu, bfu), (bcr, bfr), (bce, bfe) = (torch.split(b, S) for b in (bu, br, be))   # (:80-83)
    nz = torch.as_tensor(np.ascontiguousarray(noise[:steps]), dtype=torch.float32)
    out_c = torch.zeros(B, dtype=torch.long)                                         # (:89-90)
    out_f = torch.zeros(B, dtype=torch.long)
    hidden = torch.zeros(B, H)
    res = torch.empty(B, steps, dtype=torch.int64)
    with torch.no_grad():
        for i in range(steps):
            hc, hf = torch.split(hidden, S, dim=1)                                   # (:102-103)
            prev = torch.stack([out_c.float() / 127.5 - 1.0, out_f.float() / 127.5 - 1.0], dim=1)
            Icu, Icr, Ice = torch.split(F.linear(prev, Ic), S, dim=1)                # (:111-113)
            Rcu, Rfu, Rcr, Rfr, Rce, Rfe = torch.split(F.linear(hidden, R), S, dim=1)   # (:116-119)
            u = torch.sigmoid(Rcu + Icu + bcu)                                       # (:122-125)
            r = torch.sigmoid(Rcr + Icr + bcr)
            e = torch.tanh(r * Rce + Ice + bce)
            hc = u * hc + (1.0 - u) * e
            p = F.softmax(F.linear(F.relu(F.linear(hc, O1w, O1b)), O2w, O2b), dim=1)   # (:128-129)
            out_c = (p / nz[i, :, :Q]).argmax(dim=1)                                 # Categorical (:130-131)
            fin = torch.cat([prev, (out_c.float() / 127.5 - 1.0).unsqueeze(1)], dim=1)  # (:135-136)
            Ifu, Ifr, Ife = torch.split(F.linear(fin, If), S, dim=1)
            u = torch.sigmoid(Rfu + Ifu + bfu)                                       # (:142-145)
            r = torch.sigmoid(Rfr + Ifr + bfr)
            e = torch.tanh(r * Rfe + Ife + bfe)
            hf = u * hf + (1.0 - u) * e
            p = F.softmax(F.linear(F.relu(F.linear(hf, O3w, O3b)), O4w, O4b), dim=1)   # (:148-149)
            out_f = (p / nz[i, :, Q:]).argmax(dim=1)
            hidden = torch.cat([hc, hf], dim=1)                                      # (:154)
            res[:, i] = out_c * 256 + out_f - 2 ** 15
    return res.numpy()


def timed_deepmind(state, B: int, noise: np.ndarray, steps: int, threads: Optional[int] = None) -> dict:
    """deepmind_loop over a bounded slice of `steps` steps × B rows, wall-timed."""
    if threads:
        torch.set_num_threads(threads)
    t0 = time.perf_counter()
    out = deepmind_loop(state, B, noise, steps)
    return {"loop_s": time.perf_counter() - t0, "steps": steps, "rows": B, "out": out,
            "threads": torch.get_num_threads()}
