"""Diagnostic for the XCD-resident block-sparse kernel (fatchord_xcds.hip, rnn 896): oracle
parity under injected noise (B = 1, 3), then device µs/step of it and of the rows kernel for
8 rows (BASELINE config 4's per-GPU batch).
    python tools/diag_xcds.py [L]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.loop import FatchordLoop  # noqa: E402
from wavernn_amd.pruning import prune_state  # noqa: E402

if os.environ.get("TIME_DM_LIB"):   # A/B of two builds of the library (diagnostics only)
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]


def cond_of(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()


def main(L=6000):
    d = syn.SPARSE896_MOL
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    for B, Lp in ((1, 300), (3, 200)):
        state = prune_state(syn.make_fatchord_state(d, 3), 0.95)
        mels, aux = syn.make_conditioning(B, Lp, d.feat_dims, d.res_out_dims, 4)
        noise = syn.make_noise("MOL", B, Lp, d.n_classes, 9)
        ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
        os.environ["WRNN_PATH"] = "xcd"
        loop.set_weights(state)
        print("info", loop.info, flush=True)
        try:
            out, _ = loop.generate(cond_of(mels, aux), noise=torch.from_numpy(noise).cuda())
        except Exception as e:
            print(f"xcds parity B={B}: {e}", flush=True)
            continue
        err = np.abs(out.cpu().numpy() - ref)
        print(f"xcds parity B={B} L={Lp}: path {loop.info['last_path']} max|d| {err.max():.3g} "
              f"at {np.unravel_index(err.argmax(), err.shape)}", flush=True)
    state = prune_state(syn.make_fatchord_state(d, 5), 0.95)
    mels, aux = syn.make_conditioning(8, L, d.feat_dims, d.res_out_dims, 6)
    cond = cond_of(mels, aux)
    loop.set_weights(state)
    for rnd in range(2):
        for p in ("xcd", "rows"):
            os.environ["WRNN_PATH"] = p
            loop.generate(cond, seed=11)
            dev = min((loop.generate(cond, seed=11), loop.elapsed_ms())[1] for _ in range(3))
            print(f"round {rnd} {p} B=8: {dev * 1e3 / L:.3f} us/step ({8 * L / dev / 1e3:.3f} M samples/s), "
                  f"path {loop.info['last_path']}", flush=True)
    loop.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
