"""In-tree build of the HIP library (hipcc → wavernn_amd/_lib/libwavernn_amd.so, gfx950)."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_lib", "libwavernn_amd.so")
SOURCES = [os.path.join(CSRC, f) for f in ("fatchord_loop.hip", "fatchord_split.hip", "fatchord_xcd.hip", "fatchord_xcds.hip", "fatchord_xcdm.hip", "fatchord_rows.hip", "deepmind_rows.hip", "deepmind_xcd.hip", "condition.hip", "frame_terms.hip", "melresnet.hip", "capi.cpp")]
HEADERS = [os.path.join(CSRC, f) for f in ("fatchord_loop.h", "fatchord_split.h", "fatchord_xcd.h", "fatchord_xcds.h", "fatchord_xcdm.h", "deepmind_xcd.h", "mfma_device.h", "xcd_device.h", "fatchord_rows.h", "deepmind_rows.h", "wrnn_device.h",
                                           "rows_device.h")] + \
    [os.path.join(REPO, "include", "wavernn_amd.h")]
ARCH = os.environ.get("WRNN_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


OBJDIR = os.path.join(os.path.dirname(OUT), "obj")


def _compile_cmd(src: str) -> list:
    common = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(REPO, "include")]
    return common + EXTRA_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", _obj(src)]


def _obj(src: str) -> str:
    return os.path.join(OBJDIR, os.path.basename(src) + ".o")


def _stamp_ok(src: str) -> bool:
    """The object was compiled by exactly today's command (arch and flags included): each object
    keeps its command line in <obj>.cmd, so a changed WRNN_OFFLOAD_ARCH or flag rebuilds it."""
    try:
        with open(_obj(src) + ".cmd") as f:
            return f.read() == " ".join(_compile_cmd(src))
    except OSError:
        return False


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in SOURCES + HEADERS) and all(_stamp_ok(s) for s in SOURCES)


# per-source extra flags: the multi-row kernel's register-blocked dots are plain fp32 FMAs; the
# SLP vectorizer packs them into v_pk_fma_f32 with operand-shuffling moves and mid-loop LDS
# waits (measured 4x slower jobs on gfx950)
EXTRA_FLAGS = {"fatchord_rows.hip": ["-fno-slp-vectorize"], "fatchord_split.hip": ["-fno-slp-vectorize"],
               "fatchord_xcd.hip": ["-fno-slp-vectorize"], "fatchord_xcds.hip": ["-fno-slp-vectorize"], "fatchord_xcdm.hip": ["-fno-slp-vectorize"], "deepmind_rows.hip": ["-fno-slp-vectorize"], "deepmind_xcd.hip": ["-fno-slp-vectorize"]}


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile the sources whose object is older than the source or any header (all of them in
    parallel, one hipcc each), then link."""
    if not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    os.makedirs(OBJDIR, exist_ok=True)
    newest_header = max(os.path.getmtime(h) for h in HEADERS)
    objs, todo = [], []
    for src in SOURCES:
        obj = _obj(src)
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), newest_header) \
                or not _stamp_ok(src):
            todo.append(src)
    jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 8))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for src in todo:
            if os.path.exists(_obj(src) + ".cmd"):
                os.remove(_obj(src) + ".cmd")
            if verbose:
                print(" ".join(_compile_cmd(src)), flush=True)
        for src, f in [(src, ex.submit(subprocess.run, _compile_cmd(src), check=True)) for src in todo]:
            f.result()
            with open(_obj(src) + ".cmd", "w") as fh:
                fh.write(" ".join(_compile_cmd(src)))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-lrocblas", "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
