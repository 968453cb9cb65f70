"""Run the MoL loop with per-stage stamps (WRNN_DEBUG_STAMPS) and summarise where a step's
time goes.  Stamp k = s_memrealtime (100 MHz) at the end of stage k (see fatchord_loop.hip)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from wavernn_amd import synthetic as syn
from wavernn_amd.loop import FatchordLoop

NAMES = ["start", "gru1 + hop A (h1)", "gru2 + hop B (h2)", "fc1 + hop C (f1)", "fc2 + hop D (f2)",
         "fc3 (+hop E)", "sample + end"]
NST = len(NAMES)


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
    # skew: when do workgroups publish h1 (stamp 12) relative to the earliest, per step
    pub = st[:, :, 12]
    valid = pub > 0
    if valid.all():
        rel = (pub - pub.min(0, keepdims=True)) * 10e-3
        print(f"  h1 publish skew across WGs: median of per-step max {np.median(rel.max(0)):.3f} us")
        done = st[:, :, 1]
        lat = (done - pub.max(0, keepdims=True)) * 10e-3
        print(f"  last publish -> gather done: median {np.median(lat):.3f} us (p90 {np.percentile(lat, 90):.3f})")
        pub2 = st[:, :, 13]
        lat2 = (st[:, :, 2] - pub2.max(0, keepdims=True)) * 10e-3
        print(f"  h2 publish skew: {np.median(((pub2 - pub2.min(0, keepdims=True)) * 10e-3).max(0)):.3f} us; "
              f"last publish -> gather done: {np.median(lat2):.3f} us")
        g1 = (pub - st[:, :, 0]) * 10e-3
        g2 = (pub2 - st[:, :, 1]) * 10e-3
        print(f"  critical compute: gru1 (start->publish) {np.median(g1):.3f} us, gru2 (hop A done->publish) {np.median(g2):.3f} us")
        s9 = (st[:, :, 9] - st[:, :, 1]) * 10e-3
        s10 = (st[:, :, 10] - st[:, :, 9]) * 10e-3
        s11 = (st[:, :, 11] - st[:, :, 10]) * 10e-3
        s13 = (st[:, :, 13] - st[:, :, 11]) * 10e-3
        print(f"  gru2 detail: bar->start {np.median(s9):.3f}  row_dot {np.median(s10):.3f}  gates {np.median(s11):.3f}  publish {np.median(s13):.3f} us")
        print(f"  hop B polling: passes median {np.median(st[:, :, 14]):.1f} (p90 {np.percentile(st[:, :, 14], 90):.0f}), "
              f"first pass {np.median(st[:, :, 15]) * 10e-3:.3f} us")
        start_skew = (st[:, :, 0] - st[:, :, 0].min(0, keepdims=True)) * 10e-3
        print(f"  step-start skew across WGs: median of max {np.median(start_skew.max(0)):.3f} us")


if __name__ == "__main__":
    if sys.argv[1:] == ["quick"]:
        main("MOL", 1, 2000)
        sys.exit(0)
    main("MOL", 1, 2000)
    main("RAW", 1, 2000)

