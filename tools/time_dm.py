"""Deepmind dual-softmax kernel: device time per step for a few row counts (and, with
WRNN_ROW_GROUPS=1|2 in the environment, one or two row groups).
    python tools/time_dm.py [B ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.loop import DeepmindLoop  # noqa: E402

if os.environ.get("TIME_DM_LIB"):   # A/B of two builds of the library (diagnostics only)
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]


def main(rows):
    dm = syn.DEFAULT_DM
    loop = DeepmindLoop(dm.hidden_size, dm.quantisation)
    loop.set_weights(syn.make_deepmind_state(dm, 0))
    for B in rows:
        loop.generate(B, 100, seed=1)
        loop.generate(B, 4000, seed=2)
        ms = loop.elapsed_ms()
        print(f"path {loop.info['last_path']} groups {os.environ.get('WRNN_ROW_GROUPS', 'auto')} B={B}: "
              f"{ms * 1e3 / 4000:.2f} us/step, {B * 4000 / ms * 1e3 / 1e6:.3f} M samples/s", flush=True)
    loop.close()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [8, 32, 64])
