"""MelResNet: the fused kernel at 16- and 4-frame tiles (WRNN_MR_FRAMES) vs the torch module, one
5 s and one 60 s mel, HIP-event timed (10 calls each after a warm-up).  Also checks that the two
tile sizes agree (same summation order per output: they must be bit-identical)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wavernn_amd import condition, synthetic as syn  # noqa: E402
from wavernn_amd.fatchord_version import WaveRNN  # noqa: E402

d = syn.DEFAULT_MOL
m = WaveRNN(**d.ctor_kwargs()).cuda().eval()
m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, 0).items()})
res = m.upsample.resnet
cfg, pk = condition.melresnet_cfg(res), condition.melresnet_pack(res)


def timed(f, n=10):
    with torch.no_grad():
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            f()
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for T in (405, 4815):
    x = torch.rand(1, 80, T + 4, device='cuda')
    outs = {}
    for F in ("16", "4"):
        os.environ["WRNN_MR_FRAMES"] = F
        us = timed(lambda: condition.melresnet(cfg, pk, x))
        outs[F] = condition.melresnet(cfg, pk, x).clone()
        print(f"T={T}: kernel, {F:>2}-frame tiles {us:8.1f} us")
    os.environ.pop("WRNN_MR_FRAMES")
    print(f"T={T}: torch module (MIOpen)    {timed(lambda: res(x)):8.1f} us; default "
          f"{timed(lambda: condition.melresnet(cfg, pk, x)):8.1f} us; tiles 16 vs 4 bit-identical: "
          f"{torch.equal(outs['16'], outs['4'])}; vs module max |d| "
          f"{(outs['4'] - res(x)).abs().max().item():.2e}", flush=True)
