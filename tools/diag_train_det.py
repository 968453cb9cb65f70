"""Why does the training-backward error against the CPU vary run to run?

Runs the teacher-forced forward + backward of tests/test_gpu_training_forward.py K times on the
GPU with identical inputs and reports, per parameter, the spread of the GPU gradients between
runs (relative to the parameter's largest gradient) and the error against the CPU module —
first with default algorithms, then with torch.use_deterministic_algorithms(True) and
torch.backends.cudnn.deterministic = True (MIOpen).  A parameter whose gradient differs between
GPU runs points at the nondeterministic op; the rest of the error is summation order.

    python tools/diag_train_det.py [MOL|RAW] [K]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.fatchord_version import WaveRNN  # noqa: E402


def grads(model, x, mel):
    model.zero_grad(set_to_none=True)
    y = model(x, mel)
    y.square().mean().backward()
    return y.detach().cpu(), {n: p.grad.detach().cpu().clone() for n, p in model.named_parameters()
                              if p.grad is not None}


def main(mode="MOL", K=4):
    d = syn.DEFAULT_MOL if mode == "MOL" else syn.DEFAULT_RAW
    state = {k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, 5).items()}
    g = np.random.default_rng(3)
    B, T = 2, 4
    mel = torch.from_numpy(g.uniform(0, 1, (B, d.feat_dims, T + 2 * d.pad)).astype(np.float32))
    x = torch.from_numpy(g.uniform(-1, 1, (B, T * d.hop_length)).astype(np.float32))
    cpu = WaveRNN(**d.ctor_kwargs())
    cpu.load_state_dict(state)
    cpu.train()
    yc, gc = grads(cpu, x, mel)
    for det in (False, True):
        torch.use_deterministic_algorithms(det, warn_only=True)
        torch.backends.cudnn.deterministic = det
        torch.backends.cudnn.benchmark = False
        gpu = WaveRNN(**d.ctor_kwargs()).cuda()
        gpu.load_state_dict(state)
        gpu.train()
        runs = [grads(gpu, x.cuda(), mel.cuda()) for _ in range(K)]
        print(f"\n== {mode} deterministic={det}: forward spread between runs "
              f"{max((r[0] - runs[0][0]).abs().max().item() for r in runs):.3e}, vs CPU "
              f"{max((r[0] - yc).abs().max().item() for r in runs):.3e}")
        rows = []
        for n in gc:
            scale = gc[n].abs().max().item() + 1e-12
            spread = max((r[1][n] - runs[0][1][n]).abs().max().item() for r in runs) / scale
            vs_cpu = max((r[1][n] - gc[n]).abs().max().item() for r in runs) / scale
            rows.append((vs_cpu, spread, n))
        rows.sort(reverse=True)
        for vs_cpu, spread, n in rows[:12]:
            print(f"  {n:32s} vs CPU {vs_cpu:.2e}   GPU run-to-run spread {spread:.2e}")
        nondet = [n for _, s, n in rows if s > 0]
        print(f"  parameters whose GPU gradient differs between runs: {nondet if nondet else 'none'}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "MOL", int(sys.argv[2]) if len(sys.argv) > 2 else 4)
