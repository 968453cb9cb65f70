"""Diagnostic for the XCD-resident kernel (fatchord_xcd.hip): oracle parity under injected
noise (B = 1 and 3 rows, time-chunked too), Philox agreement with the role-split kernel, then
device µs/step of both kernels over L steps (best of 3).
    python tools/diag_xcd.py [L]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.loop import FatchordLoop  # noqa: E402


if os.environ.get("TIME_DM_LIB"):   # A/B of two builds of the library (diagnostics only)
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]


def cond_of(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()


def main(L=20000):
    d = syn.DEFAULT_MOL
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    print("info", loop.info, flush=True)
    for B, Lp, chunk in ((1, 400, None), (3, 300, None), (1, 500, "4")):
        state = syn.make_fatchord_state(d, 3)
        mels, aux = syn.make_conditioning(B, Lp, d.feat_dims, d.res_out_dims, 4)
        noise = syn.make_noise("MOL", B, Lp, d.n_classes, 9)
        ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
        os.environ["WRNN_PATH"] = "xcd"
        os.environ.pop("WRNN_TERMS_MB", None)
        if chunk:
            os.environ["WRNN_TERMS_MB"] = chunk
        loop.set_weights(state)
        try:
            out, _ = loop.generate(cond_of(mels, aux), noise=torch.from_numpy(noise).cuda())
        except Exception as e:   # a diagnostic build may abort; keep timing it
            print(f"xcd parity B={B} L={Lp}: {e}", flush=True)
            continue
        os.environ.pop("WRNN_TERMS_MB", None)
        err = np.abs(out.cpu().numpy() - ref)
        print(f"xcd parity B={B} L={Lp} chunked={bool(chunk)}: path {loop.info['last_path']} max|d| {err.max():.3g} "
              f"at {np.unravel_index(err.argmax(), err.shape)}", flush=True)
    state = syn.make_fatchord_state(d, 5)
    mels, aux = syn.make_conditioning(1, L, d.feat_dims, d.res_out_dims, 6)
    cond = cond_of(mels, aux)
    loop.set_weights(state)
    res = {}
    for rnd in range(2):
        for p in ("xcd", "split"):
            os.environ["WRNN_PATH"] = p
            res[p], _ = loop.generate(cond, seed=11)
            dev = min((loop.generate(cond, seed=11), loop.elapsed_ms())[1] for _ in range(3))
            print(f"round {rnd} {p}: {dev * 1e3 / L:.3f} us/step ({L / dev:.1f}k samples/s), path {loop.info['last_path']}",
                  flush=True)
    print(f"philox xcd vs split max|d| {(res['xcd'] - res['split']).abs().max().item():.3g}", flush=True)
    loop.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
