"""Per-stage timeline of the XCD-resident kernel (fatchord_xcd.hip) from its WRNN_DEBUG_STAMPS
(s_memrealtime, 100 MHz, wave 0 of every workgroup).  For each step, times are relative to the
earliest step start over the XCD's 32 workgroups; the table gives the median over steps of the
min / median / max over the workgroups.
    python tools/stamps_xcd.py [L] [sparse]     (sparse: the rnn-896 block-sparse kernel, fatchord_xcds.hip)
(GRU2_STAMPS=1 / BAR_STAMPS=1 with TIME_DM_LIB: the labels of those diagnostic builds)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402

if os.environ.get("TIME_DM_LIB"):   # a diagnostic build (tools/build_alt.py)
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]
from wavernn_amd.loop import FatchordLoop  # noqa: E402

SPARSE_STAMPS = [(0, "start (after B1)"), (1, "GRU1 done (after B2)"), (2, "Y published (GRU2)"),
                 (3, "w4: Y gathered"), (4, "w4: f1 published"), (5, "w1: F1 gathered"),
                 (6, "w0: F2 published (+3 hand-offs)"), (7, "F2 gathered"), (8, "sample done"),
                 (9, "w1: GH1 terms + h2 published"), (10, "w4: h2 gathered"), (11, "w5: S quarter gathered"),
                 (13, "w5: GH2 done"), (12, "w7: ring done")]
STAMPS = [(0, "start (after B1)"), (1, "GRU1 done (after B2)"), (2, "Y published (GRU2)"), (3, "w1: Y gathered"),
          (4, "w1: f1 published"), (5, "w3: F1 gathered"), (6, "w3: F2 published"), (7, "F2 gathered"),
          (8, "sample done"), (9, "w3: GH1 terms published"), (10, "w6: h2 gathered"),
          (14, "w5: S quarter gathered"), (12, "w7: ring done"), (11, "w1: S quarter + GH2 done"),
          (13, "w5: GH2 done")]


def main(L=3000, sparse=0):
    labels = dict(SPARSE_STAMPS if sparse else STAMPS)
    if os.environ.get("GRU2_STAMPS"):   # the WRNN_XCDS_GRU2_STAMPS build: slots 12..14 inside GRU2
        labels.update({12: "w0: GRU2 block-row dots", 13: "w0: GRU2 z/n exchanged", 14: "w0: GRU2 gate math"})
    if os.environ.get("BAR_STAMPS"):   # the WRNN_XCD_BAR_STAMPS build: every wave's step-end barrier arrival
        for k in (3, 9, 10, 11, 12, 13, 14):
            labels.pop(k, None)
        labels.update({9 + i: f"w{1 + i}: at the end barrier" for i in range(6)})
        labels[3] = "w7: at the end barrier"
    os.makedirs("gpurun_out", exist_ok=True)
    path = "gpurun_out/stamps_xcd.bin"
    os.environ["WRNN_DEBUG_STAMPS"] = str(L)
    os.environ["WRNN_DEBUG_FILE"] = path
    os.environ["WRNN_PATH"] = "xcd"
    d = syn.SPARSE896_MOL if sparse else syn.DEFAULT_MOL
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    state = syn.make_fatchord_state(d, 0)
    if sparse:
        from wavernn_amd.pruning import prune_state
        state = prune_state(state, 0.95)
    loop.set_weights(state)
    mels, aux = syn.make_conditioning(1, L, d.feat_dims, d.res_out_dims, 5)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
    loop.generate(cond, seed=1)
    raw = np.fromfile(path, dtype=np.uint32)
    G, S, K = raw[:3].view(np.int32)
    st = raw[3:].reshape(G, S, K).astype(np.int64)[:32, 200:S - 2]
    t0 = st[:, :, 0].min(axis=0)
    rel = (st - t0[None, :, None]) * 10e-3
    period = np.diff(t0) * 10e-3
    clk = (st[:, -1, 15] - st[:, 0, 15]) % (1 << 32) / ((st[:, -1, 0] - st[:, 0, 0]) * 10e-9) / 1e9
    print(f"xcd kernel L={L}: step period median {np.median(period):.3f} us (stamped build), "
          f"shader clock {np.median(clk):.3f} GHz (s_memtime / s_memrealtime)")
    print("-- median over steps of (min / median / max over the 32 workgroups), us")
    for k, lab in sorted(labels.items(), key=lambda kv: (kv[0] > 8, kv[0])):
        x = rel[:, :, k]
        print(f"   {lab:28s} {np.median(x.min(0)):6.2f} {np.median(np.median(x, 0)):6.2f} {np.median(x.max(0)):6.2f}")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
