"""Diagnostic for the batch-1 role-split kernel: oracle parity (injected noise), a chunked run,
and timings against the uniform latency kernel.  Optional stamps: WRNN_DEBUG_STAMPS=<steps>."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from oracle import oracle
from wavernn_amd import synthetic as syn
from wavernn_amd.loop import FatchordLoop


def make(d, L, seed):
    state = syn.make_fatchord_state(d, seed)
    mels, aux = syn.make_conditioning(1, L, d.feat_dims, d.res_out_dims, seed + 1)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
    return state, mels, aux, cond


def parity(L=400):
    d = syn.DEFAULT_MOL
    state, mels, aux, cond = make(d, L, 3)
    noise = syn.make_noise("MOL", 1, L, d.n_classes, 9)
    ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    print("info", loop.info, flush=True)
    loop.set_weights(state)
    out, _ = loop.generate(cond, noise=torch.from_numpy(noise).cuda())
    err = np.abs(out.cpu().numpy() - ref)
    print(f"split parity L={L}: path {loop.info['last_path']} max|d| {err.max():.3g} at {err.argmax()}", flush=True)
    loop.close()


def timing(path, L=5000):
    os.environ["WRNN_PATH"] = path
    d = syn.DEFAULT_MOL
    state, _, _, cond = make(d, L, 5)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    loop.set_weights(state)
    loop.generate(cond, seed=1)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        loop.generate(cond, seed=1)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t, loop.elapsed_ms()))
    wall, dev = min(ts)
    print(f"{path:8s} L={L}: device {dev * 1e3 / L:.2f} us/step ({L / dev * 1e3 / 1e3:.1f}k samples/s), "
          f"wall {wall * 1e6 / L:.2f} us/step, path {loop.info['last_path']}", flush=True)
    loop.close()
    os.environ.pop("WRNN_PATH", None)


if __name__ == "__main__":
    print(torch.cuda.get_device_name(0), flush=True)
    parity()
    timing("split")
    timing("latency")
    if len(sys.argv) > 1:
        timing("split", int(sys.argv[1]))
