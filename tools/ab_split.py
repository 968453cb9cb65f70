"""A/B timing of the batch-1 role-split kernel under environment variants, in one process.
    python tools/ab_split.py VAR=a,b [L]     e.g. WRNN_SPLIT_XCD=0,1
Each variant: oracle parity on 400 steps (injected noise), then device µs/step over L steps
(best of 3), interleaved twice so that clock drift shows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.loop import FatchordLoop  # noqa: E402
from tools.diag_split import make  # noqa: E402

if os.environ.get("TIME_DM_LIB"):   # A/B of two builds of the library (diagnostics only)
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]


def main(spec, L):
    var, vals = spec.split("=")
    d = syn.DEFAULT_MOL
    os.environ["WRNN_PATH"] = "split"
    state, mels, aux, cond = make(d, 400, 3)
    noise = syn.make_noise("MOL", 1, 400, d.n_classes, 9)
    ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
    tstate, _, _, tcond = make(d, L, 5)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    for rnd in range(2):
        for v in vals.split(","):
            os.environ[var] = v
            loop.set_weights(state)
            out, _ = loop.generate(cond, noise=torch.from_numpy(noise).cuda())
            err = float(np.abs(out.cpu().numpy() - ref).max())
            loop.set_weights(tstate)
            loop.generate(tcond, seed=1)
            dev = min((loop.generate(tcond, seed=1), loop.elapsed_ms())[1] for _ in range(3))
            print(f"round {rnd} {var}={v}: parity max|d| {err:.3g}, {dev * 1e3 / L:.3f} us/step "
                  f"({L / dev:.1f}k samples/s), path {loop.info['last_path']}", flush=True)
    loop.close()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20000)
