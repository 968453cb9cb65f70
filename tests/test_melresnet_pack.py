"""The fused MelResNet's packed weights (condition.melresnet_pack, every BatchNorm folded into its
conv) interpreted on the CPU exactly as csrc/melresnet.hip walks them, against the reference-layout
torch module in eval mode (fatchord_version.py:13-48).  The kernel itself: tests/test_gpu_melresnet.py."""
import numpy as np
import pytest
import torch

from wavernn_amd import condition
from wavernn_amd import synthetic as syn


def _module(d, seed):
    from wavernn_amd.fatchord_version import WaveRNN
    st = syn.make_fatchord_state(d, seed)
    m = WaveRNN(**d.ctor_kwargs())
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in st.items()})
    return m.upsample.resnet.eval()


def _run_packed(p, cfg, x):
    """x [U][in][T + 2pad] float64 → [U][R][T], the kernel's layer order and layouts."""
    cin, C, R, K = cfg.in_dims, cfg.compute_dims, cfg.res_out_dims, 2 * cfg.pad + 1
    U, _, Tp = x.shape
    T = Tp - K + 1
    o = 0

    def take(n):
        nonlocal o
        v = p[o:o + n]
        o += n
        return v
    W0, b0 = take(cin * K * C).reshape(cin * K, C), take(C)
    cols = np.stack([x[:, c, tap:tap + T] for c in range(cin) for tap in range(K)], 1)   # [U][cin·K][T]
    a = np.maximum(np.einsum("kc,ukt->uct", W0, cols) + b0[None, :, None], 0.0)
    for _ in range(cfg.res_blocks):
        W1, b1, W2, b2 = take(C * C).reshape(C, C), take(C), take(C * C).reshape(C, C), take(C)
        h = np.maximum(np.einsum("kc,ukt->uct", W1, a) + b1[None, :, None], 0.0)
        a = a + np.einsum("kc,ukt->uct", W2, h) + b2[None, :, None]
    Wo, bo = take(C * R).reshape(C, R), take(R)
    assert o == p.size
    return np.einsum("kr,ukt->urt", Wo, a) + bo[None, :, None]


@pytest.mark.parametrize("d", [syn.DEFAULT_MOL, syn.TINY_MOL])
def test_packed_weights_reproduce_the_module(d):
    res = _module(d, 3)
    # non-trivial running statistics (the synthetic state's are the defaults)
    g = torch.Generator().manual_seed(5)
    for mod in res.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            mod.running_mean.copy_(torch.randn(mod.num_features, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(mod.num_features, generator=g) + 0.5)
    cfg = condition.melresnet_cfg(res)
    packed = condition.melresnet_pack(res).numpy().astype(np.float64)
    x = torch.rand(2, d.feat_dims, 23 + 2 * d.pad, generator=g)
    with torch.no_grad():
        want = res(x).double().numpy()
    got = _run_packed(packed, cfg, x.double().numpy())
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * np.abs(want).max())
