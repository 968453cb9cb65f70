"""Run the MoL loop with per-stage stamps (WRNN_DEBUG_STAMPS) and summarise where a step's
time goes.  Stamp k = s_memrealtime (100 MHz) at the end of stage k (see fatchord_loop.hip)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from wavernn_amd import synthetic as syn
from wavernn_amd.loop import FatchordLoop

NAMES = ["start", "gru1 (all units)", "gru2 + hop B (h2)", "fc1 + hop C (f1)", "fc2 + hop D (f2)",
         "fc3 (+hop E)", "sample + end"]
NST = len(NAMES)
# (publish stamp, stage-done stamp, label): per-workgroup time its first item was published
HOPS = [(13, 2, "hop B (h2)"), (7, 3, "hop C (f1)"), (8, 4, "hop D (f2)")]


def main(mode="MOL", B=1, L=2000, grid=0):
    path = "gpurun_out/stamps.bin"
    os.environ["WRNN_DEBUG_STAMPS"] = str(L)
    os.environ["WRNN_DEBUG_FILE"] = path
    d = syn.DEFAULT_MOL if mode == "MOL" else syn.DEFAULT_RAW
    state = syn.make_fatchord_state(d, 0)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 5)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, grid=grid)
    loop.set_weights(state)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
    loop.generate(cond, seed=1)
    ms = loop.elapsed_ms()
    del os.environ["WRNN_DEBUG_STAMPS"]
    raw = np.fromfile(path, dtype=np.uint32)
    G, S, K = raw[:3].view(np.int32)
    st = raw[3:].reshape(G, S, K).astype(np.int64)
    st = st[:, 100:S - 1]                     # skip warm-up and the unflushed last step
    print(f"{mode} B={B} L={L} grid={G}: kernel {ms:.1f} ms = {ms * 1e3 / L:.2f} us/step (stamped build)")
    step = (st[:, 1:, 0] - st[:, :-1, 0]) * 10e-3
    print(f"step period (us): median {np.median(step):.2f}")
    for k in range(1, NST):
        dk = (st[:, :, k] - st[:, :, k - 1]) * 10e-3
        print(f"  {NAMES[k]:22s} median {np.median(dk):7.3f} us  p10 {np.percentile(dk, 10):7.3f}  p90 {np.percentile(dk, 90):7.3f}")
    for pk, dk_, label in HOPS:
        pub = st[:, :, pk]
        if not (pub > 0).all():
            continue
        skew = ((pub - pub.min(0, keepdims=True)) * 10e-3).max(0)
        lat = (st[:, :, dk_] - pub.max(0, keepdims=True)) * 10e-3
        comp = (pub - st[:, :, dk_ - 1]) * 10e-3
        print(f"  {label}: compute->publish {np.median(comp):.3f} us, publish skew {np.median(skew):.3f} us, "
              f"last publish -> all gathered {np.median(lat):.3f} us (p90 {np.percentile(lat, 90):.3f})")
    t12 = (st[:, :, 12] - st[:, :, 1]) * 10e-3
    print(f"  gru1 terms of t+1 published {np.median(t12):.3f} us after gru1 done")


if __name__ == "__main__":
    if sys.argv[1:] == ["quick"]:
        main("MOL", 1, 2000)
        sys.exit(0)
    main("MOL", 1, 2000)
    main("RAW", 1, 2000)

