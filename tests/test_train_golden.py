"""§8(f)4 on the CPU: the drop-in's teacher-forced forward (wavernn_amd.fatchord_version.WaveRNN.forward,
kept for the reference's train loop) against the REFERENCE's own forward and backward
(models/fatchord_version.py:131-167; fixtures written by tests/golden/make_golden.py train_*):
eval-mode outputs, train-mode outputs (BatchNorm batch statistics), the loss, and every
parameter's gradient (norm and first values).  Same ATen ops on the same CPU: tight bounds."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf


def run(fx, device="cpu", deterministic=False):
    from wavernn_amd.fatchord_version import WaveRNN
    d, state, mel, x = gf.train_inputs(fx)
    m = WaveRNN(**d.ctor_kwargs()).to(device)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
    xs, ms = torch.from_numpy(x).to(device), torch.from_numpy(mel).to(device)
    m.eval()
    with torch.no_grad():
        y_eval = m(xs, ms).cpu().numpy()
    m.train()
    y = m(xs, ms)
    loss = y.square().mean()
    loss.backward()
    grads = {n: p.grad.detach().cpu().numpy().astype(np.float64).ravel() for n, p in m.named_parameters()
             if p.grad is not None}
    return y_eval, y.detach().cpu().numpy(), float(loss.item()), grads


def check(fx, y_eval, y_train, loss, grads, out_tol, loss_rtol, grad_rtol):
    s = int(fx["out_stride"])
    assert np.abs(y_eval[:, ::s] - fx["y_eval"]).max() <= out_tol
    assert np.abs(y_train[:, ::s] - fx["y_train"]).max() <= out_tol
    assert abs(loss - float(fx["loss"])) <= loss_rtol * abs(float(fx["loss"]))
    names = [str(n) for n in fx["grad_names"]]
    assert sorted(names) == sorted(grads)
    worst = 0.0
    for i, n in enumerate(names):
        g = grads[n]
        scale = np.abs(g).max() + 1e-30
        k = min(g.size, fx["grad_heads"].shape[1])
        err = np.abs(g[:k] - fx["grad_heads"][i, :k]).max() / scale
        nrm = abs(np.sqrt((g * g).sum()) - fx["grad_norms"][i]) / (fx["grad_norms"][i] + 1e-30)
        worst = max(worst, err, nrm)
    assert worst <= grad_rtol, worst
    return worst


@pytest.mark.parametrize("name", gf.TRAIN_CASES)
def test_training_forward_backward_matches_reference_cpu(name):
    fx = gf.load(name)
    y_eval, y_train, loss, grads = run(fx)
    check(fx, y_eval, y_train, loss, grads, out_tol=1e-5, loss_rtol=1e-5, grad_rtol=1e-4)
