"""Loop timings (µs per step, HIP events around the launches incl. the terms GEMM) of the
many-row XCD kernel against the other fatchord kernels, MoL rnn 512, Philox noise.

    python tools/time_xcdm.py [L] [B,B,...] [paths]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.loop import FatchordLoop  # noqa: E402


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    Bs = [int(b) for b in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8, 10, 16, 32, 64, 115, 128]
    paths = sys.argv[3].split(",") if len(sys.argv) > 3 else ["xcdm", "xcd", "rows"]
    d = syn.DEFAULT_MOL
    state = syn.make_fatchord_state(d, 0)
    for B in Bs:
        mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 1)
        cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
        line = [f"B={B:4d}"]
        for p in paths:
            if p == "xcd" and B > 48:
                continue
            os.environ["WRNN_PATH"] = p
            loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
            loop.set_weights(state)
            loop.generate(cond[:200].contiguous(), seed=1)   # warm-up
            best = 1e30
            for _ in range(2):
                t0 = time.perf_counter()
                loop.generate(cond, seed=1)
                wall = time.perf_counter() - t0
                best = min(best, loop.elapsed_ms())
            line.append(f"{p} {1000 * best / L:7.3f} us/step (path {loop.info['last_path']}, wall {wall:.2f}s)")
            loop.close()
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
