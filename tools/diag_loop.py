"""Diagnostic: run the HIP loop vs the oracle on small cases and print errors/timings
(never raises on a numerical mismatch, so one GPU call shows every case)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from oracle import oracle
from wavernn_amd import synthetic as syn
from wavernn_amd.loop import FatchordLoop


def run(d, B, L, grid=0, philox=False):
    state = syn.make_fatchord_state(d, 0)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 5)
    noise = syn.make_noise(d.mode, B, L, d.n_classes, 6)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0, grid=grid)
    loop.set_weights(state)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
    nz = None if philox else torch.from_numpy(noise).cuda()
    t = time.perf_counter()
    out, lab = loop.generate(cond, noise=nz, want_labels=True, seed=5)
    wall = time.perf_counter() - t
    ms = loop.elapsed_ms()
    msg = f"{d.mode} R={d.rnn_dims} B={B} L={L} grid={loop.info['grid']} rows/launch={loop.info['max_rows']} " \
          f"lds={loop.info['lds_bytes']} | kernel {ms:.2f} ms = {ms * 1e3 / L:.2f} us/step, wall {wall * 1e3:.1f} ms"
    if not philox:
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


if __name__ == "__main__":
    print(torch.cuda.get_device_name(0), flush=True)
    run(syn.TINY_MOL, 1, 200)
    run(syn.DEFAULT_MOL, 1, 300)
    run(syn.DEFAULT_RAW, 1, 300)
    run(syn.DEFAULT_MOL, 3, 300)
    run(syn.DEFAULT_RAW, 2, 300)
    run(syn.TINY_RAW, 2, 300)
    run(syn.DEFAULT_MOL, 1, 5000)
    run(syn.DEFAULT_MOL, 1, 5000, philox=True)
    run(syn.DEFAULT_RAW, 1, 5000)
    for g in (64, 128):
        try:
            run(syn.DEFAULT_MOL, 1, 3000, grid=g)
        except Exception as e:  # grids whose slab does not fit LDS are rejected up front
            print(f"grid {g}: {e}")
