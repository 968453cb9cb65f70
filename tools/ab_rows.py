"""A/B of the multi-row kernel (WRNN_PATH=rows) under environment variants, in one process.
    python tools/ab_rows.py VAR=a,b [B ...]        e.g. WRNN_ROWS_GRANULES=0,1 2 5 10 16
Per B and variant: oracle parity on 300 steps (injected noise, MoL 512), then device µs/step
over 3000 steps (best of 3)."""
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


def main(spec, rows, L=3000):
    var, vals = spec.split("=")
    d = syn.DEFAULT_MOL
    os.environ["WRNN_PATH"] = "rows"
    state = syn.make_fatchord_state(d, 0)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    loop.set_weights(state)
    for B in rows:
        mels, aux = syn.make_conditioning(B, 300, d.feat_dims, d.res_out_dims, 3)
        noise = syn.make_noise("MOL", B, 300, d.n_classes, 9)
        ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
        pc = cond_of(mels, aux)
        tc = cond_of(*syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 5))
        for v in vals.split(","):
            os.environ[var] = v
            out, _ = loop.generate(pc, noise=torch.from_numpy(noise).cuda())
            err = float(np.abs(out.cpu().numpy() - ref).max())
            loop.generate(tc, seed=1)
            dev = min((loop.generate(tc, seed=1), loop.elapsed_ms())[1] for _ in range(3))
            print(f"B={B:3d} {var}={v}: parity max|d| {err:.3g}, {dev * 1e3 / L:.2f} us/step "
                  f"({B * L / dev / 1e3:.3f} M samples/s)", flush=True)
    loop.close()


if __name__ == "__main__":
    main(sys.argv[1], [int(a) for a in sys.argv[2:]] or [2, 10, 16])
