"""Diagnostic for the deepmind dual-softmax kernel: label parity vs the oracle, and timings."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from oracle import oracle
from wavernn_amd import synthetic as syn
from wavernn_amd.loop import DeepmindLoop


def run(d, B, L, check=True, philox=False):
    try:
        state = syn.make_deepmind_state(d, 0)
        noise = syn.make_dm_noise(B, L, d.quantisation, 6)
        loop = DeepmindLoop(d.hidden_size, d.quantisation)
        loop.set_weights(state)
        nz = None if philox else torch.from_numpy(noise).cuda()
        loop.generate(B, L, noise=nz, seed=5)
        torch.cuda.synchronize()
        t = time.perf_counter()
        out, comb = loop.generate(B, L, noise=nz, seed=5)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t
        ms = loop.elapsed_ms()
        msg = (f"DM H={d.hidden_size} B={B} L={L} grid={loop.info['grid']} | device {ms:.2f} ms = {ms * 1e3 / L:.2f} "
               f"us/step, {B * L / ms * 1e3 / 1e6:.3f} M samples/s, wall {wall * 1e3:.1f} ms")
        if check and not philox:
            c, f, o = oracle.deepmind_loop(state, B, L, noise)
            got = comb.cpu().numpy().astype(np.int64)
            eq = got == o
            msg += f" | combined equal {eq.mean():.4f} first diff {np.argwhere(~eq)[:1].tolist()}"
            msg += f" | out==combined {bool((out.cpu().numpy() == got).all())}"
        print(msg, flush=True)
        loop.close()
    except Exception as e:
        print(f"DM H={d.hidden_size} B={B} L={L}: {type(e).__name__}: {e}", flush=True)


if __name__ == "__main__":
    print(torch.cuda.get_device_name(0), flush=True)
    run(syn.TINY_DM, 1, 300)
    run(syn.TINY_DM, 5, 300)
    run(syn.DEFAULT_DM, 1, 500)
    run(syn.DEFAULT_DM, 4, 300)
    run(syn.DEFAULT_DM, 1, 3000, check=False, philox=True)
    run(syn.DEFAULT_DM, 32, 2000, check=False, philox=True)
    run(syn.DEFAULT_DM, 64, 1000, check=False, philox=True)
