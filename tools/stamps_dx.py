"""Phase timings of the XCD-resident deepmind kernel from its debug stamps (WRNN_DEBUG_STAMPS).

    python tools/stamps_dx.py B [L]

Runs one deepmind generate through the kernel with stamps on (48 steps, kept in LDS, from step 16),
then prints, per wave, the median over those steps and over workgroups of each phase boundary
relative to the step start, in shader cycles and µs (clock: stamped step vs the launch's mean)."""
import os
import subprocess
import sys

import numpy as np

NAMES = {0: "step start", 1: "coarse gates + publish h_c", 2: "h_c poll + stage + draws issued",
         3: "O1 MFMAs + barrier", 4: "O1 epilogue + publish o1", 5: "R coarse half MFMAs",
         6: "o1 poll done + staged", 7: "O2 MFMAs + barrier", 8: "O2 epilogue + publish logits",
         9: "c_t sampled + barrier", 10: "fine gates + publish h_f", 11: "h_f poll + stage",
         12: "O3 MFMAs + barrier", 13: "O3 epilogue + publish o3", 14: "R fine half MFMAs + partials",
         15: "o3 poll done + staged", 16: "O4 MFMAs + barrier", 17: "O4 epilogue + publish logits",
         18: "f_t sampled (+ output)", 19: "w0: h_c published", 20: "h_c poll starts (after vmcnt(0))"}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    path = "/tmp/dx_stamps.bin" if not os.environ.get("GRAFT_REPO_ROOT") else "gpurun_out/dx_stamps.bin"
    env = dict(os.environ, WRNN_DEBUG_STAMPS="1", WRNN_DEBUG_FILE=path)
    env.pop("WRNN_PATH", None)
    code = (
        "import os, sys; sys.path.insert(0, '.')\n"
        "from wavernn_amd import _native\n"
        "if os.environ.get('TIME_DM_LIB'): _native.LIB_PATH = os.environ['TIME_DM_LIB']\n"
        "from wavernn_amd import synthetic as syn\nfrom wavernn_amd.loop import DeepmindLoop\n"
        f"d = syn.DEFAULT_DM; B, L = {B}, {L}\n"
        "loop = DeepmindLoop(d.hidden_size, d.quantisation)\n"
        "loop.set_weights(syn.make_deepmind_state(d, 0))\n"
        "loop.generate(B, L, seed=1)\nassert loop.info['last_path'] == 8\nprint('device_ms', loop.elapsed_ms())\n")
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
    # step-start skew between the workgroups of one XCD (workgroup b sits on XCD b % 8): the
    # s_memrealtime stamp (10 ns ticks) of wave 0 at each step start, max − min over the XCD
    blk = np.nonzero(live)[0]
    skews = []
    for x in range(8):
        sel = st[(blk % 8) == x, 0, :, K - 1]
        if sel.shape[0] > 1:
            skews.append(sel.max(0) - sel.min(0))
    if skews:
        sk = np.concatenate(skews) / 100.0
        print(f"step-start skew over an XCD's workgroups: median {np.median(sk):.3f} us, 90th pct "
              f"{np.percentile(sk, 90):.3f} us, max {sk.max():.3f} us")
    # the h_c and h_f hops in real time (10 ns ticks): last publish over the XCD's workgroups (wave 0:
    # slot 22 / 23) → each wave's poll done (slot 21 / 24); each workgroup's own publish after its
    # step start; and the spread of the publishes over the XCD (last − first)
    for name, s_pub, s_done in (("h_c", 22, 21), ("h_f", 23, 24)):
        hop, own, spread = [], [], []
        for x in range(8):
            m = (blk % 8) == x
            if m.sum() < 2:
                continue
            pub = st[m, 0, :, s_pub]
            last = pub.max(0)
            spread.append(last - pub.min(0))
            for w in range(waves):
                hop.append(st[m, w, :, s_done] - last[None, :])
            own.append(pub - st[m, 0, :, K - 1])
        if hop:
            hp, ow = np.concatenate(hop).ravel() / 100.0, np.concatenate(own).ravel() / 100.0
            sp = np.concatenate(spread).ravel() / 100.0
            ok = (hp > -5) & (hp < 20)
            print(f"{name} publish after the own step start: median {np.median(ow):.3f} us, max {ow.max():.3f} us; "
                  f"spread over the XCD median {np.median(sp):.3f} us; poll done after the XCD's last publish: "
                  f"median {np.median(hp[ok]):.3f} us, 90th pct {np.percentile(hp[ok], 90):.3f} us")
    for w in range(waves):
        rel = st[:, w, :, :] - base[:, w]
        print(f"-- wave {w}")
        prev = 0.0
        for k in [k for k in range(1, K - 1) if k not in (21, 22, 23, 24)]:
            v = rel[..., k]
            v = v[(v > 0) & (v < 10 * step)]
            if v.size == 0:
                continue
            med = float(np.median(v))
            print(f"  {k:2d} {NAMES.get(k, ''):40s} {med:8.0f} cyc  (+{med - prev:6.0f})  {med / cyc_per_us:6.3f} us")
            prev = med


if __name__ == "__main__":
    main()
