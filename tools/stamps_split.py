"""Per-stage timeline of the batch-1 role-split kernel (fatchord_split.hip) from its
WRNN_DEBUG_STAMPS (s_memrealtime, 100 MHz).  For each step, times are relative to the earliest
step start over all workgroups; the table gives the median over steps of the min / median / max
over the workgroups of each role."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from wavernn_amd import synthetic as syn
from wavernn_amd.loop import FatchordLoop

GRU = [(0, "start"), (1, "GRU1 done"), (2, "Y published (GRU2 done)"), (4, "F2 partial logits gathered"),
       (5, "sample done"), (3, "phase C done")]
FC = [(0, "start"), (1, "Y gathered"), (6, "f1 published"), (2, "F1 gathered"), (3, "fc2 done"),
      (7, "partial logits published")]


def main(L=3000):
    os.makedirs("gpurun_out", exist_ok=True)
    path = "gpurun_out/stamps_split.bin"
    os.environ["WRNN_DEBUG_STAMPS"] = str(L)
    os.environ["WRNN_DEBUG_FILE"] = path
    os.environ["WRNN_PATH"] = "split"
    d = syn.DEFAULT_MOL
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    loop.set_weights(syn.make_fatchord_state(d, 0))
    mels, aux = syn.make_conditioning(1, L, d.feat_dims, d.res_out_dims, 5)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
    loop.generate(cond, seed=1)
    ms = loop.elapsed_ms()
    Gg = loop.info["split_grid"] - 512 // 16
    raw = np.fromfile(path, dtype=np.uint32)
    G, S, K = raw[:3].view(np.int32)
    st = raw[3:].reshape(G, S, K).astype(np.int64)[:, 200:S - 2]
    t0 = st[:, :, 0].min(axis=0)                       # earliest start per step
    rel = (st - t0[None, :, None]) * 10e-3             # us
    period = np.diff(t0) * 10e-3
    print(f"split kernel L={L} G={G} (GRU {Gg}, FC {G - Gg}): {ms * 1e3 / L:.2f} us/step (stamped); "
          f"step period median {np.median(period):.2f} us")
    for name, sl, stamps in (("GRU", slice(0, Gg), GRU), ("FC", slice(Gg, G), FC)):
        print(f"-- {name} workgroups: median over steps of (min / median / max over workgroups), us")
        for k, lab in stamps:
            x = rel[sl, :, k]
            print(f"   {lab:28s} {np.median(x.min(0)):6.2f} {np.median(np.median(x, 0)):6.2f} {np.median(x.max(0)):6.2f}")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
