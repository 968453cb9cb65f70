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


def noise_width(mode: str, n_classes: int) -> int:
    """K of the injected-noise layout [L][B][K] (reference draw order)."""
    return 11 if mode == "MOL" else n_classes


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
        self._create(nat.Config(nat.ABI_VERSION, nat.MODE_MOL if mode == "MOL" else nat.MODE_RAW, rnn_dims,
                                fc_dims, aux_dims, feat_dims, n_classes, grid, timeout_ms), device)

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
