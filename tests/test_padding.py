"""Dims that are not multiples of 4 (the reference constructor takes any, fatchord_version.py:93-123)
run zero-padded to the kernels' float4 layouts (wavernn_amd/loop.py:pad_loop_state).  The padding
is exact in real arithmetic (only zero terms are added); the oracle on the padded weights and
conditioning gives the same RAW labels and MoL samples within 1e-6 (its blocked dot products
re-associate when the row length changes), far inside the 1e-5 kernel tolerance."""
import numpy as np
import pytest

from oracle import oracle
from wavernn_amd import synthetic as syn
from wavernn_amd.loop import pad_loop_state


def _pad_cond(x, A, Ap):
    B, L, C = x.shape
    out = np.zeros((B, L, 4 * Ap), np.float32)
    for j in range(4):
        out[:, :, j * Ap:j * Ap + A] = x[:, :, j * A:(j + 1) * A]
    return out


@pytest.mark.parametrize("mode", ["MOL", "RAW"])
def test_padding_is_exact_in_the_oracle(mode):
    d = syn.FatchordDims(rnn_dims=30, fc_dims=37, bits=6, compute_dims=16, res_out_dims=20, res_blocks=1,
                         mode=mode)
    R, F, A, M = d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims
    assert (R % 4, F % 4, A % 4) != (0, 0, 0)
    Rp, Fp, Ap = 32, 40, (A + 3) // 4 * 4
    state = syn.make_fatchord_state(d, 11)
    B, L = 2, 120
    mels, aux = syn.make_conditioning(B, L, M, d.res_out_dims, 12)
    noise = syn.make_noise(mode, B, L, d.n_classes, 13)
    ref, ref_lab = oracle.fatchord_loop(state, mode, mels, aux, noise)
    ps = pad_loop_state(state, R, F, A, M, Rp, Fp, Ap)
    assert ps["rnn2.weight_ih_l0"].shape == (3 * Rp, Rp + Ap) and ps["fc3.weight"].shape[1] == Fp
    out, lab = oracle.fatchord_loop(ps, mode, mels, _pad_cond(aux, A, Ap), noise)
    assert np.abs(out - ref).max() <= 1e-6
    if mode == "RAW":
        np.testing.assert_array_equal(lab, ref_lab)
