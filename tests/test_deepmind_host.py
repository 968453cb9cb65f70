"""Host-side checks of the deepmind drop-in (no GPU): reference parameter names/shapes, the
training forward, and that generate() refuses to run on the CPU (no fallback)."""
import numpy as np
import pytest
import torch

from wavernn_amd import synthetic as syn
from wavernn_amd.deepmind_version import WaveRNN
from wavernn_amd.loop import DM_KEYS


def test_state_dict_matches_reference_layout():
    d = syn.TINY_DM
    m = WaveRNN(**d.ctor_kwargs())
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert shapes == {k: tuple(s) for k, s in syn.deepmind_state_shapes(d).items()}
    assert set(DM_KEYS) == set(shapes)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in syn.make_deepmind_state(d, 0).items()}, strict=True)


def test_forward_matches_a_numpy_restatement():
    """deepmind_version.py:37-72 step, restated in numpy (fp64) on the same weights."""
    d = syn.TINY_DM
    st = syn.make_deepmind_state(d, 3)
    m = WaveRNN(**d.ctor_kwargs())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    g = np.random.default_rng(0)
    prev_y = g.uniform(-1, 1, (2, 2)).astype(np.float32)
    h = g.uniform(-1, 1, (2, d.hidden_size)).astype(np.float32)
    cc = g.uniform(-1, 1, (2, 1)).astype(np.float32)
    oc, of, hn = m(torch.from_numpy(prev_y), torch.from_numpy(h), torch.from_numpy(cc))
    S = d.split_size
    f64 = {k: v.astype(np.float64) for k, v in st.items()}
    R = h @ f64["R.weight"].T
    Ic = prev_y @ f64["I_coarse.weight"].T
    If = np.concatenate([prev_y, cc], 1) @ f64["I_fine.weight"].T
    I = [np.concatenate([Ic[:, i * S:(i + 1) * S], If[:, i * S:(i + 1) * S]], 1) for i in range(3)]
    H = d.hidden_size
    sig = lambda x: 1 / (1 + np.exp(-x))
    u = sig(R[:, :H] + I[0] + f64["bias_u"])
    r = sig(R[:, H:2 * H] + I[1] + f64["bias_r"])
    e = np.tanh(r * R[:, 2 * H:] + I[2] + f64["bias_e"])
    hid = u * h + (1 - u) * e
    relu = lambda x: np.maximum(x, 0)
    o_c = relu(hid[:, :S] @ f64["O1.weight"].T + f64["O1.bias"]) @ f64["O2.weight"].T + f64["O2.bias"]
    o_f = relu(hid[:, S:] @ f64["O3.weight"].T + f64["O3.bias"]) @ f64["O4.weight"].T + f64["O4.bias"]
    np.testing.assert_allclose(hn.detach().numpy(), hid, atol=1e-5)
    np.testing.assert_allclose(oc.detach().numpy(), o_c, atol=1e-4)
    np.testing.assert_allclose(of.detach().numpy(), o_f, atol=1e-4)


def test_generate_has_no_cpu_fallback():
    m = WaveRNN(**syn.TINY_DM.ctor_kwargs())
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.generate(10)
