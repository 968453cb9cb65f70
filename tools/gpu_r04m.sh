#!/bin/bash
# Round 4: fused MelResNet with weight loads issued 16 ahead — parity + A/B vs the torch module.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_melresnet.py -q --timeout 200 --timeout-method thread > gpurun_out/mr_pt2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/mr_pt2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_frames.py 3 b1 fold60s > gpurun_out/ab_mr2.log 2>&1 || exit $?
grep -E "x RT" gpurun_out/ab_mr2.log
timeout -k 10 120 python -u - <<'PY' 2>&1 | grep -v amdgpu.ids
import sys, time, torch, numpy as np
sys.path.insert(0, '.')
from wavernn_amd import synthetic as syn, condition
from wavernn_amd.fatchord_version import WaveRNN
d = syn.DEFAULT_MOL
m = WaveRNN(**d.ctor_kwargs()).cuda().eval()
m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, 0).items()})
res = m.upsample.resnet
cfg, pk = condition.melresnet_cfg(res), condition.melresnet_pack(res)
for T in (405, 4814):
    x = torch.rand(1, 80, T + 4, device='cuda')
    for name, f in (("kernel", lambda: condition.melresnet(cfg, pk, x)), ("torch", lambda: res(x))):
        with torch.no_grad():
            f(); torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): f()
            e1.record(); torch.cuda.synchronize()
        print(f"T={T} {name}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per MelResNet")
PY
