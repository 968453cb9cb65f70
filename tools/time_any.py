"""Loop timings (µs per step, HIP events around the launches incl. the terms GEMM) for any
fatchord dims and kernel paths, Philox noise.

    python tools/time_any.py --mode RAW --rnn 512 --fc 512 --L 2000 --B 1,2,10 --paths ,latency,rows

An empty path name is the library's default choice for that row count."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.loop import FatchordLoop  # noqa: E402

if os.environ.get("TIME_DM_LIB"):   # A/B of two builds of the library (diagnostics only)
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="MOL")
    ap.add_argument("--rnn", type=int, default=512)
    ap.add_argument("--fc", type=int, default=512)
    ap.add_argument("--L", type=int, default=2000)
    ap.add_argument("--B", default="1")
    ap.add_argument("--paths", default="")
    ap.add_argument("--prune", type=float, default=0.0)
    args = ap.parse_args()
    d = syn.FatchordDims(rnn_dims=args.rnn, fc_dims=args.fc, mode=args.mode)
    state = syn.make_fatchord_state(d, 0)
    if args.prune > 0:
        from wavernn_amd.pruning import prune_state
        state = prune_state(state, args.prune)
    L = args.L
    for B in [int(b) for b in args.B.split(",")]:
        mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 1)
        cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
        line = [f"{args.mode} rnn {args.rnn} fc {args.fc} B={B:4d}"]
        for p in args.paths.split(","):
            os.environ["WRNN_PATH"] = p
            loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
            loop.set_weights(state)
            loop.generate(cond[:100].contiguous(), seed=1)   # warm-up
            best = 1e30
            for _ in range(2):
                t0 = time.perf_counter()
                loop.generate(cond, seed=1, want_labels=args.mode == "RAW")
                wall = time.perf_counter() - t0
                best = min(best, loop.elapsed_ms())
            line.append(f"[{p or 'default'}] {1000 * best / L:8.3f} us/step (path {loop.info['last_path']}, "
                        f"wall {wall:.2f}s)")
            loop.close()
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
