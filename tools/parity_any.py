"""Parity of a library build (TIME_DM_LIB, A/B builds) against the C oracle under injected noise,
for MoL row counts (rnn 512, or --rnn 896 --prune 0.95 for the block-sparse kernel) on a forced path — the check an alternative build must pass before its
timings count.   TIME_DM_LIB=tools/_alt/x.so python tools/parity_any.py --B 10,32 --L 300 --path xcdm"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402

if os.environ.get("TIME_DM_LIB"):
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", default="10")
    ap.add_argument("--L", type=int, default=300)
    ap.add_argument("--path", default="xcdm")
    ap.add_argument("--rnn", type=int, default=512)
    ap.add_argument("--prune", type=float, default=0.0)
    args = ap.parse_args()
    from oracle import oracle
    from wavernn_amd.loop import FatchordLoop
    os.environ["WRNN_PATH"] = args.path
    d = syn.FatchordDims(rnn_dims=args.rnn, fc_dims=512, mode="MOL")
    worst = 0.0
    for B in [int(b) for b in args.B.split(",")]:
        state = syn.make_fatchord_state(d, 700 + B)
        if args.prune > 0:
            from wavernn_amd.pruning import prune_state
            state = prune_state(state, args.prune)
        mels, aux = syn.make_conditioning(B, args.L, d.feat_dims, d.res_out_dims, 701 + B)
        noise = syn.make_noise("MOL", B, args.L, d.n_classes, 702 + B)
        ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
        loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
        loop.set_weights(state)
        cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
        out, _ = loop.generate(cond, noise=torch.from_numpy(noise).cuda())
        err = float(np.abs(out.cpu().numpy() - ref).max())
        worst = max(worst, err)
        print(f"B={B} L={args.L} path {loop.info['last_path']}: max |d| vs oracle {err:.3g}", flush=True)
        loop.close()
    print("PARITY OK" if worst <= 1e-5 else "PARITY FAIL", flush=True)
    sys.exit(0 if worst <= 1e-5 else 1)


if __name__ == "__main__":
    main()
