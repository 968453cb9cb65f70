import os, sys, time
sys.path.insert(0, ".")
import torch
from wavernn_amd import synthetic as syn
from wavernn_amd.loop import DeepmindLoop
dm = syn.DEFAULT_DM
for g in ("1", "2"):
    os.environ["WRNN_ROW_GROUPS"] = g
    loop = DeepmindLoop(dm.hidden_size, dm.quantisation)
    loop.set_weights(syn.make_deepmind_state(dm, 0))
    for B in (8, 32, 64):
        loop.generate(B, 100, seed=1)
        loop.generate(B, 4000, seed=2)
        ms = loop.elapsed_ms()
        print(f"groups {g} B={B}: {ms * 1e3 / 4000:.2f} us/step, {B * 4000 / ms * 1e3 / 1e6:.3f} M samples/s", flush=True)
    loop.close()
