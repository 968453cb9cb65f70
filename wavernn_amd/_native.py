"""ctypes binding of the C-ABI (include/wavernn_amd.h) in libwavernn_amd.so.

The product path has no fallback: if the HIP library is missing or cannot be loaded this
module raises, it never substitutes a CPU implementation."""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_lib", "libwavernn_amd.so")

ABI_VERSION = 6
MODE_RAW, MODE_MOL, MODE_DM = 0, 1, 2
STATUS = {0: "WRNN_OK", -1: "WRNN_EINVAL", -2: "WRNN_EHIP", -3: "WRNN_ENOWEIGHTS", -4: "WRNN_ETIMEOUT",
          -5: "WRNN_ENOMEM", -6: "WRNN_EUNSUPPORTED"}

# Every symbol include/wavernn_amd.h declares (tests check the .so exports all of them).
EXPORTS = ("wrnn_create", "wrnn_set_weights", "wrnn_generate", "wrnn_check", "wrnn_elapsed_ms",
           "wrnn_query", "wrnn_last_error", "wrnn_destroy", "wrnn_cond_shape", "wrnn_upsample_pack",
           "wrnn_postprocess", "wrnn_cond_last_error", "wrnn_generate_frames", "wrnn_generate_frames_rows",
           "wrnn_frame_weights", "wrnn_melresnet_floats", "wrnn_melresnet", "wrnn_philox_draws",
           "wrnn_melresnet_tile_frames")


class MelResNetCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("in_dims", "compute_dims", "res_out_dims", "res_blocks", "pad")]


class WrnnError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("abi_version", "mode", "rnn_dims", "fc_dims", "aux_dims",
                                              "feat_dims", "n_classes", "grid", "timeout_ms")]


class Tensor(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("numel", ctypes.c_int64),
                ("on_device", ctypes.c_int32)]


class Info(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("grid", "units_rnn", "units_fc", "units_cls", "max_rows",
                                              "lds_bytes", "slab_floats", "num_cus", "rows_grid",
                                              "rows_units_rnn", "sparse_blocks", "split_grid", "last_path",
                                              "xcd_rows", "xcdm_rows")]


class UpsampleCfg(ctypes.Structure):
    _fields_ = [("feat_dims", ctypes.c_int32), ("res_out_dims", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("n_scales", ctypes.c_int32), ("scales", ctypes.c_int32 * 4),
                ("taps", ctypes.POINTER(ctypes.c_float) * 4)]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libwavernn_amd.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build the HIP extension with "
                          "`python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
    L.wrnn_create.argtypes = [ctypes.POINTER(Config), i32, ctypes.POINTER(vp)]
    L.wrnn_create.restype = i32
    L.wrnn_set_weights.argtypes = [vp, ctypes.POINTER(Tensor), i32]
    L.wrnn_set_weights.restype = i32
    L.wrnn_generate.argtypes = [vp, vp, i32, i32, vp, u64, i64, vp, vp, vp]
    L.wrnn_generate.restype = i32
    L.wrnn_check.argtypes = [vp, vp]
    L.wrnn_check.restype = i32
    L.wrnn_elapsed_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.wrnn_elapsed_ms.restype = i32
    L.wrnn_query.argtypes = [vp, ctypes.POINTER(Info)]
    L.wrnn_query.restype = i32
    L.wrnn_last_error.argtypes = [vp]
    L.wrnn_last_error.restype = ctypes.c_char_p
    L.wrnn_destroy.argtypes = [vp]
    L.wrnn_destroy.restype = None
    pi = ctypes.POINTER(ctypes.c_int)
    L.wrnn_cond_shape.argtypes = [ctypes.POINTER(UpsampleCfg), i32, i32, i32, i32, pi, pi]
    L.wrnn_cond_shape.restype = i32
    L.wrnn_upsample_pack.argtypes = [ctypes.POINTER(UpsampleCfg), vp, vp, i32, i32, i32, i32, vp, vp]
    L.wrnn_upsample_pack.restype = i32
    L.wrnn_postprocess.argtypes = [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp]
    L.wrnn_postprocess.restype = i32
    L.wrnn_generate_frames.argtypes = [vp, ctypes.POINTER(UpsampleCfg), vp, vp, i32, i32, i32, i32, vp, u64, i64, vp,
                                       vp, vp]
    L.wrnn_generate_frames.restype = i32
    L.wrnn_generate_frames_rows.argtypes = [vp, ctypes.POINTER(UpsampleCfg), vp, vp, i32, i32, i32, i32, i32, i32, vp,
                                            u64, i64, vp, vp, vp]
    L.wrnn_generate_frames_rows.restype = i32
    L.wrnn_frame_weights.argtypes = [ctypes.POINTER(UpsampleCfg), pi, pi, pi, vp, i32]
    L.wrnn_frame_weights.restype = i32
    L.wrnn_melresnet_floats.argtypes = [ctypes.POINTER(MelResNetCfg)]
    L.wrnn_melresnet_floats.restype = i32
    L.wrnn_melresnet.argtypes = [ctypes.POINTER(MelResNetCfg), vp, vp, i32, i32, vp, vp]
    L.wrnn_melresnet.restype = i32
    L.wrnn_melresnet_tile_frames.argtypes = [ctypes.POINTER(MelResNetCfg), i32, i32]
    L.wrnn_melresnet_tile_frames.restype = i32
    L.wrnn_philox_draws.argtypes = [u64, i64, i32, i32, i32, i32, i32, vp, vp]
    L.wrnn_philox_draws.restype = i32
    L.wrnn_cond_last_error.argtypes = []
    L.wrnn_cond_last_error.restype = ctypes.c_char_p
    _lib = L
    return L


def check_cond(code: int):
    """Status of a stateless conditioning / post-processing call."""
    if code != 0:
        raise WrnnError(code, (lib().wrnn_cond_last_error() or b"").decode(errors="replace"))


def check(handle, code: int):
    if code != 0:
        msg = lib().wrnn_last_error(handle) if handle else b""
        raise WrnnError(code, (msg or b"").decode(errors="replace"))
