"""§8(f)4: the training-side teacher-forced forward (models/fatchord_version.py:131-167;
deepmind_version.py:36-72) runs on the MI355X with the GRUs on MIOpen (torch.nn.GRU on ROCm) —
forward (1e-4) and backward (1.5e-3 of each parameter's largest gradient) against the same module
on the CPU (ATen): fp32 tolerances for the different kernels' summation orders.

The backward runs with deterministic algorithms (torch.use_deterministic_algorithms +
cudnn.deterministic, i.e. MIOpen's deterministic kernels).  Round 4 widened the bound to 5e-3
after one red run; tools/diag_train_det.py found why the error moved from run to run
(profiles/r05_train_determinism_*.log): with default algorithms the only gradients that differ
between two identical GPU runs are those of the UpsampleNetwork's box convolutions
(upsample.up_layers.{1,3,5}.weight: MIOpen's backward-weights reduction), and the algorithm
MIOpen / the BLAS pick also moves the summation order of the rest (fc1.weight 2.3e-3 of its largest
gradient under default algorithms, below 3.6e-4 deterministic).  Deterministic: two runs are
bit-identical and the largest error is 8.6e-4 (MoL fc2.weight) / 4.7e-4 (RAW fc2.weight)."""
import numpy as np
import pytest
import torch

from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _pair(d, seed):
    from wavernn_amd.fatchord_version import WaveRNN
    state = {k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, seed).items()}
    cpu = WaveRNN(**d.ctor_kwargs())
    cpu.load_state_dict(state)
    gpu = WaveRNN(**d.ctor_kwargs()).to(DEV)
    gpu.load_state_dict(state)
    return cpu, gpu


@pytest.fixture
def deterministic():
    prev = (torch.are_deterministic_algorithms_enabled(), torch.backends.cudnn.deterministic,
            torch.backends.cudnn.benchmark)
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    yield
    torch.use_deterministic_algorithms(prev[0])
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev[1], prev[2]


@pytest.mark.parametrize("mode", ["MOL", "RAW"])
def test_fatchord_training_forward_backward_on_miopen(mode, deterministic):
    d = syn.DEFAULT_MOL if mode == "MOL" else syn.DEFAULT_RAW
    cpu, gpu = _pair(d, 5)
    cpu.eval()
    gpu.eval()
    g = np.random.default_rng(3)
    B, T = 2, 4
    mel = torch.from_numpy(g.uniform(0, 1, (B, d.feat_dims, T + 2 * d.pad)).astype(np.float32))
    x = torch.from_numpy(g.uniform(-1, 1, (B, T * d.hop_length)).astype(np.float32))
    yc = cpu(x, mel)
    yg = gpu(x.to(DEV), mel.to(DEV))
    assert yg.shape == yc.shape
    assert (yg.detach().cpu() - yc.detach()).abs().max().item() <= 1e-4
    # backward through MIOpen's GRU (training mode: BatchNorm on batch statistics in both)
    cpu.train()
    gpu.train()
    yc = cpu(x, mel)
    yg = gpu(x.to(DEV), mel.to(DEV))
    assert (yg.detach().cpu() - yc.detach()).abs().max().item() <= 1e-4
    yc.square().mean().backward()
    yg.square().mean().backward()
    # deterministic algorithms: a second GPU backward reproduces every gradient bit for bit
    g1 = {n: p.grad.detach().clone() for n, p in gpu.named_parameters() if p.grad is not None}
    gpu.zero_grad(set_to_none=True)
    gpu(x.to(DEV), mel.to(DEV)).square().mean().backward()
    for n, p in gpu.named_parameters():
        if n in g1:
            assert torch.equal(p.grad, g1[n]), f"{n}: GPU gradient differs between two identical runs"
    rel = {}
    for (n, pc), (_, pg) in zip(cpu.named_parameters(), gpu.named_parameters()):
        if pc.grad is None:
            continue
        err = (pg.grad.cpu() - pc.grad).abs().max().item()
        rel[n] = err / (pc.grad.abs().max().item() + 1e-12)
    worst = sorted(rel, key=rel.get)[-3:]
    print(f"\n{mode}: largest relative gradient errors " + ", ".join(f"{n} {rel[n]:.2e}" for n in worst))
    # reductions over B·T = 2 200 rows in other orders (cancelling sums: the error relative to a
    # parameter's largest gradient is far above fp32 epsilon): 8.6e-4 / 4.7e-4 observed under
    # deterministic algorithms (module docstring) — a wrong backward is off by O(1)
    assert rel[worst[-1]] <= 1.5e-3, worst


def test_deepmind_training_forward_on_gpu():
    from wavernn_amd.deepmind_version import WaveRNN
    d = syn.DEFAULT_DM
    state = {k: torch.from_numpy(np.array(v)) for k, v in syn.make_deepmind_state(d, 6).items()}
    cpu = WaveRNN(**d.ctor_kwargs())
    cpu.load_state_dict(state)
    gpu = WaveRNN(**d.ctor_kwargs()).to(DEV)
    gpu.load_state_dict(state)
    g = np.random.default_rng(4)
    prev_y = torch.from_numpy(g.uniform(-1, 1, (3, 2)).astype(np.float32))
    prev_hidden = torch.from_numpy(g.uniform(-1, 1, (3, d.hidden_size)).astype(np.float32))
    current_coarse = torch.from_numpy(g.uniform(-1, 1, (3, 1)).astype(np.float32))
    outc = cpu(prev_y, prev_hidden, current_coarse)
    outg = gpu(prev_y.to(DEV), prev_hidden.to(DEV), current_coarse.to(DEV))
    for a, b in zip(outc, outg):
        assert (b.detach().cpu() - a.detach()).abs().max().item() <= 1e-5


@pytest.mark.parametrize("name", ["train_mol", "train_raw"])
def test_training_forward_backward_on_miopen_vs_reference(name, deterministic):
    """The same forward + backward on the MI355X (MIOpen GRU, deterministic algorithms) against the
    REFERENCE's own CPU outputs and gradients (tests/golden train_* fixtures): eval and train
    outputs within 1e-4, the loss within 1e-4 relative, each gradient's first values and norm
    within 1.5e-3 of its largest |value| / its norm (the bound of the CPU-module test above)."""
    from tests.golden import fixtures as gf
    from tests.test_train_golden import check, run
    fx = gf.load(name)
    y_eval, y_train, loss, grads = run(fx, device=DEV)
    worst = check(fx, y_eval, y_train, loss, grads, out_tol=1e-4, loss_rtol=1e-4, grad_rtol=1.5e-3)
    print(f"\n{name}: largest relative gradient error vs the reference {worst:.2e}")
