"""Per-row divergence of the many-row XCD kernel vs the oracle: first step over tolerance, per
launch row (XCD k = row % 8, its row n = row // 8 there).   python tools/diag_xcdm.py B [L] [seed]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.loop import FatchordLoop  # noqa: E402

if os.environ.get("TIME_DM_LIB"):   # a build under A/B (diagnostics only)
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 115
L = int(sys.argv[2]) if len(sys.argv) > 2 else 200
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 815
os.environ["WRNN_PATH"] = "xcdm"
d = syn.DEFAULT_MOL
state = syn.make_fatchord_state(d, seed)
mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, seed + 1)
noise = syn.make_noise("MOL", B, L, d.n_classes, seed + 2)
ref, _ = oracle.fatchord_loop(state, "MOL", mels, aux, noise)
loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
loop.set_weights(state)
cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
for rep in range(2):
    out, _ = loop.generate(cond, noise=torch.from_numpy(noise).cuda())
    err = np.abs(out.cpu().numpy() - ref)
    bad = [(r, int(np.argmax(err[r] > 1e-5))) for r in range(B) if err[r].max() > 1e-5]
    print(f"rep {rep}: max {err.max():.3g}; {len(bad)} rows bad:",
          " ".join(f"{r}(k{r % 8},n{r // 8})@{s}" for r, s in bad[:40]), flush=True)
