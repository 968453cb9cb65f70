"""time_dm.py plus a digest of the labels (same digest across builds = bit-identical labels)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from wavernn_amd import _native  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.loop import DeepmindLoop  # noqa: E402

if os.environ.get("TIME_DM_LIB"):
    _native.LIB_PATH = os.environ["TIME_DM_LIB"]

dm = syn.DEFAULT_DM
loop = DeepmindLoop(dm.hidden_size, dm.quantisation)
loop.set_weights(syn.make_deepmind_state(dm, 0))
for B in [int(a) for a in sys.argv[1:]] or [8, 32]:
    _, lab = loop.generate(B, 600, seed=7)
    dg = hashlib.sha1(lab.cpu().numpy().tobytes()).hexdigest()[:12]
    loop.generate(B, 4000, seed=2)
    ms = loop.elapsed_ms()
    print(f"B={B}: {ms * 1e3 / 4000:.3f} us/step digest {dg}", flush=True)
loop.close()
