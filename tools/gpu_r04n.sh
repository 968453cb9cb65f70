#!/bin/bash
# Round 4: MelResNet kernel with LDS-staged weights — parity, timing, drop-in A/B, smoke.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_melresnet.py tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread > gpurun_out/mr_pt3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/mr_pt3.log; grep -E "^FAILED|^E  " gpurun_out/mr_pt3.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u - <<'PY' 2>&1 | grep -v amdgpu.ids
import sys, torch, numpy as np
sys.path.insert(0, '.')
from wavernn_amd import synthetic as syn, condition
from wavernn_amd.fatchord_version import WaveRNN
d = syn.DEFAULT_MOL
m = WaveRNN(**d.ctor_kwargs()).cuda().eval()
m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, 0).items()})
res = m.upsample.resnet
cfg, pk = condition.melresnet_cfg(res), condition.melresnet_pack(res)
for U, T in ((1, 405), (8, 405), (1, 4814)):
    x = torch.rand(U, 80, T + 4, device='cuda')
    for name, f in (("kernel", lambda: condition.melresnet(cfg, pk, x)), ("torch", lambda: res(x))):
        with torch.no_grad():
            f(); torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): f()
            e1.record(); torch.cuda.synchronize()
        print(f"U={U} T={T} {name}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per MelResNet")
PY
timeout -k 10 400 python -u tools/ab_frames.py 3 b1 fold60s > gpurun_out/ab_mr3.log 2>&1 || exit $?
grep -E "x RT" gpurun_out/ab_mr3.log
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke3.log 2>&1 || { tail -5 gpurun_out/smoke3.log; exit 1; }
tail -1 gpurun_out/smoke3.log
