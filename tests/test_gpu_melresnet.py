"""wrnn_melresnet (csrc/melresnet.hip, the whole MelResNet in one kernel with the BatchNorms folded)
against the reference-layout torch module in eval mode on the same GPU (MIOpen), and the drop-in's
use of it.  Reference: fatchord_version.py:13-48, :183-186."""
import numpy as np
import pytest
import torch

from wavernn_amd import condition
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(d, seed):
    from wavernn_amd.fatchord_version import WaveRNN
    st = syn.make_fatchord_state(d, seed)
    m = WaveRNN(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in st.items()})
    return m.eval()


@pytest.mark.parametrize("d,U,T,F", [(syn.DEFAULT_MOL, 1, 405, 4), (syn.DEFAULT_MOL, 3, 37, 4),
                                     (syn.TINY_MOL, 2, 50, 4), (syn.DEFAULT_MOL, 1, 4815, 16)])
def test_kernel_matches_the_module(d, U, T, F):
    """F: the tile form the kernel takes for this grid on a 256-CU MI355X (4-frame tiles when the
    16-frame grid has fewer workgroups than CUs)."""
    m = _model(d, 4)
    res = m.upsample.resnet
    g = torch.Generator().manual_seed(9)
    for mod in res.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            mod.running_mean.copy_(torch.randn(mod.num_features, generator=g).to(DEV) * 0.1)
            mod.running_var.copy_((torch.rand(mod.num_features, generator=g) + 0.5).to(DEV))
    x = torch.rand(U, d.feat_dims, T + 2 * d.pad, generator=g).to(DEV)
    with torch.no_grad():
        want = res(x)
    import ctypes
    from wavernn_amd import _native as nat
    cfg = condition.melresnet_cfg(res)
    assert torch.cuda.get_device_properties(DEV).multi_processor_count == 256
    assert nat.lib().wrnn_melresnet_tile_frames(ctypes.byref(cfg), U, T) == F
    got = condition.melresnet(cfg, condition.melresnet_pack(res), x)
    err = float((got - want).abs().max())
    print(f"max |Δ| {err:.3g} of {float(want.abs().max()):.3g}")
    assert got.shape == want.shape and err <= 1e-5 * float(want.abs().max())


def test_dropin_frames_use_the_kernel_and_refresh_on_new_weights():
    m = _model(syn.DEFAULT_MOL, 5)
    mel = torch.from_numpy(syn.make_mel(80, 30, 3))[None].to(DEV)
    _, aux, _ = m.frames(mel)
    padded = m.pad_tensor(mel.transpose(1, 2), pad=m.pad, side='both').transpose(1, 2)
    with torch.no_grad():
        want = m.upsample.resnet(padded)
    assert float((aux - want).abs().max()) <= 1e-5 * float(want.abs().max())
    with torch.no_grad():
        m.upsample.resnet.conv_out.bias.add_(1.0)          # the packed copy must follow the module
    _, aux2, _ = m.frames(mel)
    assert torch.allclose(aux2, aux + 1.0, atol=1e-4)
