"""Phase timings of the many-row XCD kernel from its debug stamps (WRNN_DEBUG_STAMPS).

    python tools/stamps_xcdm.py B [L]

Runs one MoL generate through the kernel with stamps on (48 steps, kept in LDS, from step 16),
then prints, per wave, the median over those steps and over workgroups of each phase boundary
relative to the step start, in shader cycles and µs (clock: stamped step vs the launch's mean)."""
import os
import subprocess
import sys

import numpy as np

NAMES = {0: "step start", 1: "A  GRU1 + publish h1", 2: "B  h1 poll done", 3: "B  W_ih2 MFMAs + partials",
         4: "   barrier B2", 5: "C  GRU2 gate math + publish y, h2", 6: "D  W_hh1 MFMAs",
         7: "E  y poll done", 8: "E  fc1 MFMAs", 9: "   barrier B3", 10: "F  fc1 epilogue + publish f1",
         11: "G  h2 poll done", 12: "G  W_hh2 MFMAs", 13: "H  f1 poll done", 14: "H  fc2 MFMAs",
         15: "   barrier B4", 16: "I  ring loads issued + fc2 epilogue", 17: "   barrier B5",
         18: "   fc3 partials published", 19: "   ring store (two-level)", 20: "J  sampled",
         21: "   ring store (direct)"}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    path = "/tmp/xcdm_stamps.bin" if not os.environ.get("GRAFT_REPO_ROOT") else "gpurun_out/xcdm_stamps.bin"
    env = dict(os.environ, WRNN_DEBUG_STAMPS="1", WRNN_DEBUG_FILE=path, WRNN_PATH="xcdm")
    code = (
        "import numpy as np, torch, sys; sys.path.insert(0, '.')\n"
        "from wavernn_amd import synthetic as syn\nfrom wavernn_amd.loop import FatchordLoop\n"
        f"d = syn.DEFAULT_MOL; B, L = {B}, {L}\n"
        "loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)\n"
        "loop.set_weights(syn.make_fatchord_state(d, 0))\n"
        "m, a = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 1)\n"
        "cond = torch.from_numpy(np.concatenate([m, a], 2).transpose(1, 0, 2).copy()).cuda()\n"
        "loop.generate(cond, seed=1)\nprint('device_ms', loop.elapsed_ms())\n")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    ms = float(out.split()[-1])
    raw = np.fromfile(path, dtype=np.int32)
    G, S, K = raw[:3]
    st = raw[3:].view(np.uint32).reshape(G, S, K).astype(np.int64)
    waves = 4
    st = st.reshape(G // waves, waves, S, K)
    live = st[:, 0, 5, 0] != 0                       # workgroups of XCDs that had rows
    st = st[live]
    base = st[:, :, :, 0:1]
    step = np.median(np.diff(st[:, 0, :, 0], axis=1))
    real = np.median(np.diff(st[:, 0, :, K - 1], axis=1))   # s_memrealtime (100 MHz) at step start
    cyc_per_us = step / (real / 100.0)
    print(f"B={B}: {live.sum()} workgroups, median stamped step {step:.0f} cycles = {real / 100:.3f} us "
          f"(shader clock {cyc_per_us / 1e3:.2f} GHz); launch incl. the stamp dump {ms * 1e3 / L:.3f} us/step")
    for w in range(waves):
        rel = st[:, w, :, :] - base[:, w]
        print(f"-- wave {w}")
        prev = 0.0
        for k in range(1, K - 1):
            v = rel[..., k]
            v = v[(v > 0) & (v < 10 * step)]
            if v.size == 0:
                continue
            med = float(np.median(v))
            print(f"  {k:2d} {NAMES.get(k, ''):40s} {med:8.0f} cyc  (+{med - prev:6.0f})  {med / cyc_per_us:6.3f} us")
            prev = med


if __name__ == "__main__":
    main()
