"""A/B of the drop-in generate() with the conditioning terms formed at frame rate (default) vs the
per-sample route (WRNN_NO_FRAME_TERMS=1): wall clock per call (synchronised), best of N, for the
BASELINE shapes that run the XCD-resident kernels.
    python tools/ab_frames.py [reps] [case ...]     cases: b1 many8 fold5s fold60s sparse8"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.pruning import prune_state  # noqa: E402
from wavernn_amd.fatchord_version import WaveRNN  # noqa: E402

DEV = torch.device("cuda", 0)


def model(d, prune=0.0):
    st = syn.make_fatchord_state(d, 0)
    if prune:
        st = prune_state(st, prune)
    m = WaveRNN(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in st.items()})
    return m


def run(case, m):
    f5 = syn.frames_for_seconds(5.0)
    mel = lambda T, s=1: torch.from_numpy(syn.make_mel(80, T, s))[None]   # noqa: E731
    if case == "b1":
        return lambda: m.generate(mel(f5), None, False, 11000, 550, False, seed=1, verbose=False), f5 * 275
    if case == "many8" or case == "sparse8":
        ms = [mel(f5, 10 + i) for i in range(8)]
        return lambda: m.generate_many(ms, None, False, 11000, 550, False, seed=1), 8 * f5 * 275
    if case == "fold5s":
        return lambda: m.generate(mel(f5), None, True, 11000, 550, False, seed=1, verbose=False), f5 * 275
    if case == "fold60s":
        f60 = syn.frames_for_seconds(60.0)
        return lambda: m.generate(mel(f60), None, True, 11000, 550, False, seed=1, verbose=False), f60 * 275
    raise ValueError(case)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    cases = sys.argv[2:] or ["b1", "many8", "fold5s", "fold60s", "sparse8"]
    dense, sparse = None, None
    for case in cases:
        if case == "sparse8":
            sparse = sparse or model(syn.SPARSE896_MOL, 0.95)
            m = sparse
        else:
            dense = dense or model(syn.DEFAULT_MOL)
            m = dense
        fn, samples = run(case, m)
        modes = ("frames", "torch-melresnet", "per-sample", "frames") if not os.environ.get("AB_ONLY") \
            else (os.environ["AB_ONLY"],)
        for mode in modes:
            os.environ.pop("WRNN_NO_FRAME_TERMS", None)
            os.environ.pop("WRNN_TORCH_MELRESNET", None)
            if mode == "per-sample":
                os.environ["WRNN_NO_FRAME_TERMS"] = "1"
            elif mode == "torch-melresnet":   # MelResNet through the torch module (MIOpen), not the fused kernel
                os.environ["WRNN_TORCH_MELRESNET"] = "1"
            fn()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t)
            print(f"{case:8s} {mode:10s} {best * 1e3:9.2f} ms  {samples / best / 1e6:7.3f} M samples/s  "
                  f"{samples / best / 22050:7.1f}x RT  path {m.loop_handle().info['last_path']}", flush=True)


if __name__ == "__main__":
    main()
