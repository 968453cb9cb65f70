"""Diagnostic for the multi-row kernel (WRNN_PATH=rows): parity vs the oracle on small cases,
time-chunked launches (WRNN_TERMS_MB), and timings at fold-batched sizes.  Never raises on a
numerical mismatch, so one GPU call shows every case."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from oracle import oracle
from wavernn_amd import synthetic as syn
from wavernn_amd.loop import FatchordLoop


def run(d, B, L, check=True, philox=False, terms_mb=None, path="rows", prune=None, sparse=None):
    os.environ["WRNN_PATH"] = path
    if terms_mb:
        os.environ["WRNN_TERMS_MB"] = str(terms_mb)
    if sparse is not None:
        os.environ["WRNN_SPARSE"] = str(sparse)
    try:
        state = syn.make_fatchord_state(d, 0)
        if prune:
            from wavernn_amd.pruning import prune_state
            state = prune_state(state, prune)
        mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 5)
        noise = syn.make_noise(d.mode, B, L, d.n_classes, 6)
        loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
        loop.set_weights(state)
        cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
        nz = None if philox else torch.from_numpy(noise).cuda()
        loop.generate(cond, noise=nz, want_labels=True, seed=5)     # warm (rocBLAS init, allocations)
        torch.cuda.synchronize()
        t = time.perf_counter()
        out, lab = loop.generate(cond, noise=nz, want_labels=True, seed=5)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t
        ms = loop.elapsed_ms()
        msg = (f"{path:7s} {d.mode} R={d.rnn_dims} B={B} L={L} terms_mb={terms_mb} prune={prune} "
               f"grid={loop.info['grid']} | device {ms:.2f} ms = "
               f"{ms * 1e3 / L:.2f} us/step, {B * L / ms * 1e3 / 1e6:.3f} M samples/s, wall {wall * 1e3:.1f} ms")
        if check and not philox:
            ref, ref_lab = oracle.fatchord_loop(state, d.mode, mels, aux, noise)
            o = out.cpu().numpy()
            if d.mode == "MOL":
                e = np.abs(o - ref)
                msg += f" | max|d| {e.max():.3g} first>1e-5 {int(np.argmax(e.max(0) > 1e-5)) if (e > 1e-5).any() else -1}"
            else:
                eq = lab.cpu().numpy() == ref_lab
                msg += f" | labels equal {eq.mean():.4f} first diff {np.argwhere(~eq)[:1].tolist()}"
        print(msg, flush=True)
        loop.close()
    except Exception as e:  # report and continue
        print(f"{path} {d.mode} B={B} L={L}: {type(e).__name__}: {e}", flush=True)
    finally:
        os.environ.pop("WRNN_PATH", None)
        os.environ.pop("WRNN_TERMS_MB", None)
        os.environ.pop("WRNN_SPARSE", None)


if __name__ == "__main__":
    print(torch.cuda.get_device_name(0), flush=True)
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "dense"):
        run(syn.TINY_RAW, 2, 200)
        run(syn.TINY_MOL, 3, 200)
        run(syn.DEFAULT_MOL, 1, 200)
        run(syn.DEFAULT_RAW, 2, 200)
        run(syn.DEFAULT_MOL, 10, 300)
        run(syn.DEFAULT_MOL, 10, 300, terms_mb=20)          # several time chunks (carried state)
        run(syn.DEFAULT_RAW, 20, 200)
        run(syn.TINY_MOL, 40, 100)
        run(syn.DEFAULT_MOL, 10, 4000, check=False, philox=True)
        run(syn.DEFAULT_MOL, 32, 2000, check=False, philox=True)
        run(syn.DEFAULT_MOL, 115, 1000, check=False, philox=True)
    if which in ("all", "sparse"):
        run(syn.DEFAULT_MOL, 3, 300, prune=0.95)              # sparse rows kernel, rnn 512 (G = 128)
        run(syn.DEFAULT_MOL, 3, 300, prune=0.95, sparse=0)    # same weights, dense rows kernel
        run(syn.DEFAULT_RAW, 3, 300, prune=0.95)
        run(syn.TINY_RAW, 5, 200, prune=0.9)
        run(syn.SPARSE896_MOL, 8, 200, prune=0.95)            # config 4 dims
        run(syn.SPARSE896_MOL, 8, 3000, prune=0.95, check=False, philox=True)
        run(syn.SPARSE896_MOL, 1, 3000, prune=0.95, check=False, philox=True)
