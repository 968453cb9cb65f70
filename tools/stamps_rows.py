"""Per-stage timing of the multi-row kernel (WRNN_PATH=rows, WRNN_DEBUG_STAMPS).
Stamp k = s_memrealtime (100 MHz) at the points marked RSTAMP(k) in fatchord_rows.hip."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from wavernn_amd import synthetic as syn
from wavernn_amd.loop import FatchordLoop

SEG = [(0, 1, "gru1 + store drain + signal h1"), (1, 2, "(loader prefetch)"), (2, 3, "wait h1 + gru2 tiles + signal h2"),
       (3, 4, "off-critical (GH1, V1h)"), (4, 6, "wait h2 + fc1 tiles + signal f1"),
       (6, 7, "off-critical (GH2)"), (7, 9, "wait f1 + fc2 tiles + signal f2"),
       (9, 10, "[sampler] wait f2/logits flags"), (10, 11, "[sampler] dma + fc3 + sample"),
       (9, 12, "x hand-off (all)"), (0, 12, "step"),
       (4, 13, "  fc1: flags + first tile DMA"), (13, 14, "  fc1: jobs"), (14, 15, "  fc1: store drain")]


def main(mode="MOL", B=10, L=2000):
    path = "gpurun_out/stamps_rows.bin"
    os.environ.update(WRNN_PATH="rows", WRNN_DEBUG_STAMPS=str(L), WRNN_DEBUG_FILE=path)
    d = syn.DEFAULT_MOL if mode == "MOL" else syn.DEFAULT_RAW
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    loop.set_weights(syn.make_fatchord_state(d, 0))
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 5)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
    loop.generate(cond, seed=1)
    ms = loop.elapsed_ms()
    for k in ("WRNN_PATH", "WRNN_DEBUG_STAMPS", "WRNN_DEBUG_FILE"):
        del os.environ[k]
    raw = np.fromfile(path, dtype=np.uint32)
    G, S, K = raw[:3].view(np.int32)
    st = raw[3:].reshape(G, S, K).astype(np.int64)[:, 50:S - 1]
    print(f"{mode} B={B} L={L} grid={G}: {ms * 1e3 / L:.2f} us/step incl. terms GEMM (stamped build)")
    for k, name in ((5, "  fc1: compute wave 0 busy (sum)"), (8, "  fc1: lead loader DMA (sum)")):
        v = st[:, :, k].ravel() * 10e-3
        if (v > 0).any():
            print(f"  {name:34s} median {np.median(v[v > 0]):7.3f} us")
    for a, b, name in SEG:
        m = (st[:, :, a] > 0) & (st[:, :, b] > 0)
        if not m.any():
            continue
        dk = (st[:, :, b] - st[:, :, a])[m] * 10e-3
        print(f"  {name:34s} median {np.median(dk):7.3f} us  p10 {np.percentile(dk, 10):7.3f}  p90 {np.percentile(dk, 90):7.3f}")


if __name__ == "__main__":
    # python tools/stamps_rows.py [MODE B L]...   (default: MOL 115 400, MOL 32 1000, MOL 10 1000)
    args = sys.argv[1:] or ["MOL", "115", "400", "MOL", "32", "1000", "MOL", "10", "1000"]
    for i in range(0, len(args), 3):
        main(args[i], int(args[i + 1]), int(args[i + 2]))
