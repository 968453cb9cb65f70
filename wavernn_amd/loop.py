"""Python handle on the persistent HIP sample loop (C-ABI in include/wavernn_amd.h).

`FatchordLoop` is the device-side replacement for the per-step loop of
`WaveRNN.generate()` (models/fatchord_version.py:192-241 in the reference): one call runs
all L steps for B rows in a single persistent-kernel launch per row chunk.
"""
from __future__ import annotations

import ctypes
from typing import Mapping, Optional, Tuple

import numpy as np
import torch

from . import _native as nat

LOOP_KEYS = ("I.weight", "I.bias", "rnn1.weight_ih_l0", "rnn1.weight_hh_l0", "rnn1.bias_ih_l0",
             "rnn1.bias_hh_l0", "rnn2.weight_ih_l0", "rnn2.weight_hh_l0", "rnn2.bias_ih_l0",
             "rnn2.bias_hh_l0", "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "fc3.weight",
             "fc3.bias")


DM_KEYS = ("R.weight", "O1.weight", "O1.bias", "O2.weight", "O2.bias", "O3.weight", "O3.bias", "O4.weight",
           "O4.bias", "I_coarse.weight", "I_fine.weight", "bias_u", "bias_r", "bias_e")


def _round4(n: int) -> int:
    return (n + 3) // 4 * 4


def pad_loop_state(state: Mapping[str, np.ndarray], R: int, F: int, A: int, M: int, Rp: int, Fp: int,
                   Ap: int) -> dict:
    """Zero-pad the loop tensors of a WaveRNN with rnn / fc / aux dims R, F, A to Rp, Fp, Ap (the
    kernels' float4 layouts need multiples of 4).  Exact: a padded GRU unit has zero weights and
    biases, so r = z = ½, n = tanh(0) = 0 and h' = h / 2 stays 0 from h = 0; a padded fc row is
    relu(0) = 0; every padded column multiplies such a zero (or a zero-padded aux channel), so the
    real units, rows and logits see only added zero terms (fatchord_version.py:97-123 shapes)."""
    def gates(w, rows, rows_p, cols_map, ncols_p):
        out = np.zeros((3 * rows_p, ncols_p), np.float32)
        for g in range(3):
            for (c0, c1, d0) in cols_map:
                out[g * rows_p:g * rows_p + rows, d0:d0 + c1 - c0] = w[g * rows:(g + 1) * rows, c0:c1]
        return out

    def vec3(b, n, n_p):
        out = np.zeros(3 * n_p, np.float32)
        for g in range(3):
            out[g * n_p:g * n_p + n] = b[g * n:(g + 1) * n]
        return out

    def mat(w, rows_p, cols_map, ncols_p):
        out = np.zeros((rows_p, ncols_p), np.float32)
        for (c0, c1, d0) in cols_map:
            out[:w.shape[0], d0:d0 + c1 - c0] = w[:, c0:c1]
        return out

    def vec(b, n_p):
        out = np.zeros(n_p, np.float32)
        out[:b.shape[0]] = b
        return out

    st = {k: np.asarray(v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else v, np.float32)
          for k, v in state.items() if k in LOOP_KEYS}
    o = dict(st)
    o["I.weight"] = mat(st["I.weight"], Rp, [(0, 1 + M, 0), (1 + M, 1 + M + A, 1 + M)], 1 + M + Ap)
    o["I.bias"] = vec(st["I.bias"], Rp)
    for k in ("rnn1.weight_ih_l0", "rnn1.weight_hh_l0", "rnn2.weight_hh_l0"):
        o[k] = gates(st[k], R, Rp, [(0, R, 0)], Rp)
    o["rnn2.weight_ih_l0"] = gates(st["rnn2.weight_ih_l0"], R, Rp, [(0, R, 0), (R, R + A, Rp)], Rp + Ap)
    for k in ("rnn1.bias_ih_l0", "rnn1.bias_hh_l0", "rnn2.bias_ih_l0", "rnn2.bias_hh_l0"):
        o[k] = vec3(st[k], R, Rp)
    o["fc1.weight"] = mat(st["fc1.weight"], Fp, [(0, R, 0), (R, R + A, Rp)], Rp + Ap)
    o["fc1.bias"] = vec(st["fc1.bias"], Fp)
    o["fc2.weight"] = mat(st["fc2.weight"], Fp, [(0, F, 0), (F, F + A, Fp)], Fp + Ap)
    o["fc2.bias"] = vec(st["fc2.bias"], Fp)
    o["fc3.weight"] = mat(st["fc3.weight"], st["fc3.weight"].shape[0], [(0, F, 0)], Fp)
    return o


def noise_width(mode: str, n_classes: int) -> int:
    """K of the injected-noise layout [L][B][K] (reference draw order)."""
    return 11 if mode == "MOL" else n_classes


def philox_draws(seed: int, row_offset: int, rows: int, steps: int, K: int, mode: str, step0: int = 0,
                 device: int = 0, stream=None) -> torch.Tensor:
    """The draws a loop launch takes with noise=None (C-ABI wrnn_philox_draws): [steps][rows][K]
    fp32 on cuda:`device`, row j keyed row_offset + j, step s keyed step0 + s — usable as the
    `noise` of the same launch (bit-identical audio).  mode "MOL": U(1e-5, 1 − 1e-5) (K = 11);
    "RAW" / "DM": Exp(1)."""
    m = {"RAW": nat.MODE_RAW, "MOL": nat.MODE_MOL, "DM": nat.MODE_DM}[mode]
    dev = torch.device("cuda", device)
    out = torch.empty(steps, rows, K, dtype=torch.float32, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    rc = nat.lib().wrnn_philox_draws(ctypes.c_uint64(seed & (2 ** 64 - 1)), row_offset, rows, step0, steps, K, m,
                                     out.data_ptr(), stream)
    if rc != 0:
        raise nat.WrnnError(rc, nat.lib().wrnn_cond_last_error().decode())
    return out


class FatchordLoop:
    keys = LOOP_KEYS

    def __init__(self, mode: str, rnn_dims: int, fc_dims: int, aux_dims: int, feat_dims: int,
                 n_classes: int, device: int = 0, grid: int = 0, timeout_ms: int = 0):
        if mode not in ("RAW", "MOL"):
            raise RuntimeError("Unknown model mode value - ", mode)
        self.mode, self.rnn_dims, self.fc_dims = mode, rnn_dims, fc_dims
        self.aux_dims, self.feat_dims, self.n_classes = aux_dims, feat_dims, n_classes
        self.device = device
        self.cond_dims = feat_dims + 4 * aux_dims
        self.noise_k = noise_width(mode, n_classes)
        # dims that are not multiples of 4 run zero-padded (pad_loop_state; exact)
        self._dims_p = (_round4(rnn_dims), _round4(fc_dims), _round4(aux_dims))
        self._padded = self._dims_p != (rnn_dims, fc_dims, aux_dims)
        Rp, Fp, Ap = self._dims_p
        self._create(nat.Config(nat.ABI_VERSION, nat.MODE_MOL if mode == "MOL" else nat.MODE_RAW, Rp,
                                Fp, Ap, feat_dims, n_classes, grid, timeout_ms), device)

    def _create(self, cfg, device: int) -> None:
        L = nat.lib()
        h = ctypes.c_void_p()
        rc = L.wrnn_create(ctypes.byref(cfg), device, ctypes.byref(h))
        self._h = h
        if rc != 0:
            msg = L.wrnn_last_error(h) if h else b""
            if h:
                L.wrnn_destroy(h)
            self._h = None
            raise nat.WrnnError(rc, (msg or b"").decode())

    # ------------------------------------------------------------------ weights
    def set_weights(self, state: Mapping[str, object]) -> None:
        """Pack the loop's tensors (reference state_dict names) into the kernel layout."""
        if getattr(self, "_padded", False):
            state = pad_loop_state(state, self.rnn_dims, self.fc_dims, self.aux_dims, self.feat_dims, *self._dims_p)
        keep = []
        arr = (nat.Tensor * len(self.keys))()
        n = 0
        for k in self.keys:
            if k not in state:
                raise KeyError(f"missing weight {k!r}")
            v = state[k]
            if isinstance(v, torch.Tensor):
                v = v.detach()
                if v.is_cuda:
                    v = v.to(torch.float32).contiguous()
                    keep.append(v)
                    arr[n] = nat.Tensor(k.encode(), v.data_ptr(), v.numel(), 1)
                    n += 1
                    continue
                v = v.cpu().numpy()
            a = np.ascontiguousarray(v, dtype=np.float32)
            keep.append(a)
            arr[n] = nat.Tensor(k.encode(), a.ctypes.data, a.size, 0)
            n += 1
        nat.check(self._h, nat.lib().wrnn_set_weights(self._h, arr, n))

    # --------------------------------------------------------------------- run
    def generate(self, cond: torch.Tensor, noise: Optional[torch.Tensor] = None, seed: int = 0,
                 row_offset: int = 0, want_labels: bool = False, stream=None,
                 out: Optional[torch.Tensor] = None, labels: Optional[torch.Tensor] = None,
                 check: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """cond [L][B][feat+4·aux] fp32 on this GPU → samples [B][L] (+ labels [B][L] for RAW)."""
        if not (cond.is_cuda and cond.dtype == torch.float32 and cond.is_contiguous()):
            raise ValueError("cond must be a contiguous fp32 CUDA tensor [L][B][C]")
        L, B, C = cond.shape
        if C != self.cond_dims:
            raise ValueError(f"cond has {C} features, expected {self.cond_dims}")
        if getattr(self, "_padded", False) and self._dims_p[2] != self.aux_dims:   # aux chunks a1..a4 zero-padded
            A, Ap, M = self.aux_dims, self._dims_p[2], self.feat_dims
            cp = torch.zeros(L, B, M + 4 * Ap, dtype=cond.dtype, device=cond.device)
            cp[:, :, :M] = cond[:, :, :M]
            for j in range(4):
                cp[:, :, M + j * Ap:M + j * Ap + A] = cond[:, :, M + j * A:M + (j + 1) * A]
            cond = cp
        if noise is not None:
            if not (noise.is_cuda and noise.dtype == torch.float32 and noise.is_contiguous()):
                raise ValueError("noise must be a contiguous fp32 CUDA tensor [L][B][K]")
            if tuple(noise.shape) != (L, B, self.noise_k):
                raise ValueError(f"noise shape {tuple(noise.shape)} != {(L, B, self.noise_k)}")
        if out is None:
            out = torch.empty(B, L, dtype=torch.float32, device=cond.device)
        if want_labels and labels is None and self.mode == "RAW":
            labels = torch.empty(B, L, dtype=torch.int32, device=cond.device)
        if stream is None:
            stream = torch.cuda.current_stream(cond.device).cuda_stream
        rc = nat.lib().wrnn_generate(self._h, cond.data_ptr(), B, L,
                                     noise.data_ptr() if noise is not None else None,
                                     ctypes.c_uint64(seed & (2 ** 64 - 1)), row_offset, out.data_ptr(),
                                     labels.data_ptr() if labels is not None else None, stream)
        nat.check(self._h, rc)
        if check:
            self.check(stream)
        return out, labels

    def generate_frames(self, spec, mel: torch.Tensor, aux: torch.Tensor, target: int = 0, overlap: int = 0,
                        noise: Optional[torch.Tensor] = None, seed: int = 0, row_offset: Optional[int] = None,
                        want_labels: bool = False, stream=None, check: bool = True,
                        rows: Optional[Tuple[int, int]] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """The loop from the generate() inputs at frame rate (C-ABI wrnn_generate_frames):
        mel [U][feat][T], aux [U][4·aux][T] (MelResNet of the padded mel) fp32 on this GPU, with
        `spec` the UpsampleNetwork's condition.UpsampleSpec → samples [rows][steps] (+ labels),
        rows / steps as condition.upsample_pack would lay them out (target <= 0: unbatched).
        `rows=(begin, count)`: only those rows of the launch (wrnn_generate_frames_rows; e.g. a
        block of one utterance's folds), keyed row_offset + j.  row_offset=None keys launch row
        j as its place in the whole launch (begin + j), so a block reproduces the same rows of
        the whole launch; pass the global row id of `begin` when the launch is itself a shard."""
        for name, t in (("mel", mel), ("aux", aux)):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.dim() == 3):
                raise ValueError(f"{name} must be a contiguous fp32 CUDA tensor [U][C][T]")
        U, feat, T = mel.shape
        if feat != self.feat_dims or tuple(aux.shape) != (U, 4 * self.aux_dims, T):
            raise ValueError(f"mel {tuple(mel.shape)} / aux {tuple(aux.shape)} do not match the loop dims")
        if getattr(self, "_padded", False) and self._dims_p[2] != self.aux_dims:   # aux quarters zero-padded
            A, Ap = self.aux_dims, self._dims_p[2]
            ap = torch.zeros(U, 4 * Ap, T, dtype=aux.dtype, device=aux.device)
            for j in range(4):
                ap[:, j * Ap:j * Ap + A] = aux[:, j * A:(j + 1) * A]
            aux = ap
            spec = spec.with_res_out(4 * Ap)
        steps, n_rows = spec.shape(U, T, target, overlap)
        r0, rows = (0, n_rows) if rows is None else (int(rows[0]), int(rows[1]))
        if r0 < 0 or rows < 1 or r0 + rows > n_rows:
            raise ValueError(f"rows [{r0}, {r0 + rows}) outside the launch's {n_rows}")
        if row_offset is None:
            row_offset = r0
        if noise is not None:
            if not (noise.is_cuda and noise.dtype == torch.float32 and noise.is_contiguous()):
                raise ValueError("noise must be a contiguous fp32 CUDA tensor [L][B][K]")
            if tuple(noise.shape) != (steps, rows, self.noise_k):
                raise ValueError(f"noise shape {tuple(noise.shape)} != {(steps, rows, self.noise_k)}")
        out = torch.empty(rows, steps, dtype=torch.float32, device=mel.device)
        labels = None
        if want_labels and self.mode == "RAW":
            labels = torch.empty(rows, steps, dtype=torch.int32, device=mel.device)
        if stream is None:
            stream = torch.cuda.current_stream(mel.device).cuda_stream
        rc = nat.lib().wrnn_generate_frames_rows(self._h, ctypes.byref(spec.cfg), mel.data_ptr(), aux.data_ptr(), U,
                                                 T, target, overlap, r0, rows,
                                                 noise.data_ptr() if noise is not None else None,
                                                 ctypes.c_uint64(seed & (2 ** 64 - 1)), row_offset, out.data_ptr(),
                                                 labels.data_ptr() if labels is not None else None, stream)
        nat.check(self._h, rc)
        if check:
            self.check(stream)
        return out, labels

    def check(self, stream=None) -> None:
        """Synchronise and raise if the persistent kernel aborted (timeout)."""
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        nat.check(self._h, nat.lib().wrnn_check(self._h, stream))

    def elapsed_ms(self) -> float:
        """Device time of the persistent loop launch(es) of the last generate() (HIP events)."""
        ms = ctypes.c_float()
        nat.check(self._h, nat.lib().wrnn_elapsed_ms(self._h, ctypes.byref(ms)))
        return float(ms.value)

    @property
    def info(self) -> dict:
        i = nat.Info()
        nat.check(self._h, nat.lib().wrnn_query(self._h, ctypes.byref(i)))
        return {f: getattr(i, f) for f, _ in nat.Info._fields_}

    def close(self) -> None:
        if getattr(self, "_h", None):
            nat.lib().wrnn_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeepmindLoop(FatchordLoop):
    """Handle on the dual-softmax kernels replacing the per-step loop of
    models/deepmind_version.py:generate (:98-156) for B independent rows: deepmind_xcd.hip
    (hidden 896 / quantisation 256: 4 rows per XCD, 32 per launch, info["last_path"] 8) or
    deepmind_rows.hip (other dims, or WRNN_PATH=rows: path 3)."""
    keys = DM_KEYS

    def __init__(self, hidden_size: int = 896, quantisation: int = 256, device: int = 0, grid: int = 0,
                 timeout_ms: int = 0):
        self.mode, self.hidden_size, self.n_classes = "DM", hidden_size, quantisation
        self.device = device
        self.noise_k = 2 * quantisation
        self._create(nat.Config(nat.ABI_VERSION, nat.MODE_DM, hidden_size, 0, 0, 0, quantisation, grid, timeout_ms),
                     device)

    def generate(self, B: int, L: int, noise: Optional[torch.Tensor] = None, seed: int = 0, row_offset: int = 0,
                 stream=None, check: bool = True,
                 device: Optional[torch.device] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """→ (samples [B][L] fp32, combined int32 [B][L]): coarse·256 + fine − 2^15 per step."""
        dev = device or torch.device("cuda", self.device)
        if noise is not None:
            if not (noise.is_cuda and noise.dtype == torch.float32 and noise.is_contiguous()):
                raise ValueError("noise must be a contiguous fp32 CUDA tensor [L][B][2Q]")
            if tuple(noise.shape) != (L, B, self.noise_k):
                raise ValueError(f"noise shape {tuple(noise.shape)} != {(L, B, self.noise_k)}")
        out = torch.empty(B, L, dtype=torch.float32, device=dev)
        labels = torch.empty(B, L, dtype=torch.int32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        rc = nat.lib().wrnn_generate(self._h, None, B, L, noise.data_ptr() if noise is not None else None,
                                     ctypes.c_uint64(seed & (2 ** 64 - 1)), row_offset, out.data_ptr(),
                                     labels.data_ptr(), stream)
        nat.check(self._h, rc)
        if check:
            self.check(stream)
        return out, labels
