"""Models whose dense loop weights exceed the grid's LDS (the reference constructor accepts any
dims, models/fatchord_version.py:93-129): the multi-row kernel with its weight slab streamed from
HBM (fatchord_rows.hip, GW = true; wrnn_info.last_path 9), against the C oracle through the C-ABI.

Tolerance: MoL samples |Δ| <= MOL_TOL (1e-5) per sample under injected noise; RAW labels
bit-exact."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
DENSE896_RAW = syn.FatchordDims(rnn_dims=896, mode="RAW")
WIDE_MOL = syn.FatchordDims(rnn_dims=1024, fc_dims=768, mode="MOL")


def _loop(d):
    from wavernn_amd.loop import FatchordLoop
    return FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


def _case(d, B, L, seed):
    from oracle import oracle
    state = syn.make_fatchord_state(d, seed)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, seed + 1)
    noise = syn.make_noise(d.mode, B, L, d.n_classes, seed + 2)
    ref, labels = oracle.fatchord_loop(state, d.mode, mels, aux, noise)
    return state, mels, aux, noise, ref, labels


@pytest.mark.parametrize("B,L", [(1, 300), (3, 200), (9, 100)])
def test_dense_896_mol_vs_oracle(B, L, monkeypatch):
    """Dense (unpruned) rnn 896: 32 MB of loop weights, more than 256 × 160 KB of LDS can hold
    beside the row state — the streamed-weights kernel, every row against the oracle."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.SPARSE896_MOL
    state, mels, aux, noise, ref, _ = _case(d, B, L, 700 + B)
    loop = _loop(d)
    loop.set_weights(state)
    assert loop.info["xcd_rows"] == 0 and loop.info["rows_grid"] > 0, loop.info
    out, _ = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 9
    err = np.abs(out.cpu().numpy() - ref)
    assert err.max() <= gf.MOL_TOL, f"max |Δ| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


def test_dense_896_raw_labels_bit_exact(monkeypatch):
    """RAW 9-bit at rnn 896 dense: the 512-class softmax sample, labels bit-exact."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = DENSE896_RAW
    state, mels, aux, noise, ref, labels = _case(d, 2, 200, 720)
    loop = _loop(d)
    loop.set_weights(state)
    out, lab = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=True)
    assert loop.info["last_path"] == 9
    np.testing.assert_array_equal(lab.cpu().numpy(), labels)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_wide_mol_time_chunks(monkeypatch):
    """rnn 1024 / fc 768 (dims no shipped kernel is specialised for), time-chunked launches with
    the state carried through HBM: the oracle, and a single launch under Philox."""
    d = WIDE_MOL
    state, mels, aux, noise, ref, _ = _case(d, 2, 300, 730)
    loop = _loop(d)
    loop.set_weights(state)
    cond = _cond(mels, aux)
    whole, _ = loop.generate(cond, seed=4)
    monkeypatch.setenv("WRNN_TERMS_MB", "4")
    out, _ = loop.generate(cond, noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 9
    assert np.abs(out.cpu().numpy() - ref).max() <= gf.MOL_TOL
    chunked, _ = loop.generate(cond, seed=4)
    assert (chunked - whole).abs().max().item() <= 2 * gf.MOL_TOL


def test_deepmind_streamed_weights_bit_exact():
    """deepmind hidden 2048: 6·4·2048 floats of R rows per workgroup exceed LDS, so the slab is
    streamed (deepmind_rows.hip, GW = true; path 10); coarse/fine labels bit-exact vs the oracle."""
    from oracle import oracle
    from wavernn_amd.loop import DeepmindLoop
    d = syn.DeepmindDims(hidden_size=2048, quantisation=256)
    B, L = 2, 60
    state = syn.make_deepmind_state(d, 740)
    noise = syn.make_dm_noise(B, L, d.quantisation, 741)
    _, _, ref = oracle.deepmind_loop(state, B, L, noise)
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(state)
    out, comb = loop.generate(B, L, noise=torch.from_numpy(noise).to(DEV))
    assert loop.info["last_path"] == 10
    np.testing.assert_array_equal(comb.cpu().numpy().astype(np.int64), ref)


@pytest.mark.parametrize("mode", ["MOL", "RAW"])
def test_dims_not_multiple_of_4(mode, monkeypatch):
    """rnn 30 / fc 37 / aux 5 (res_out 20): the host handle zero-pads to 32 / 40 / 8 (exact,
    tests/test_padding.py) — MoL within MOL_TOL and RAW labels bit-exact vs the oracle on the
    original dims, at 1 and 3 rows."""
    from oracle import oracle
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.FatchordDims(rnn_dims=30, fc_dims=37, bits=6, compute_dims=16, res_out_dims=20, res_blocks=1, mode=mode)
    state = syn.make_fatchord_state(d, 750)
    for B in (1, 3):
        mels, aux = syn.make_conditioning(B, 200, d.feat_dims, d.res_out_dims, 751 + B)
        noise = syn.make_noise(mode, B, 200, d.n_classes, 753 + B)
        ref, ref_lab = oracle.fatchord_loop(state, mode, mels, aux, noise)
        loop = _loop(d)
        loop.set_weights(state)
        out, lab = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=True)
        if mode == "RAW":
            np.testing.assert_array_equal(lab.cpu().numpy(), ref_lab)
        else:
            assert np.abs(out.cpu().numpy() - ref).max() <= gf.MOL_TOL
        loop.close()


def test_dims_not_multiple_of_4_dropin_generate():
    """The same odd dims through the drop-in WaveRNN.generate() (upsample, fold, loop, post): the
    reference output length (T − 1)·hop (fatchord_version.py:184, :257) of finite samples in [−1, 1]."""
    from wavernn_amd.fatchord_version import WaveRNN
    d = syn.FatchordDims(rnn_dims=30, fc_dims=37, bits=9, compute_dims=16, res_out_dims=20, res_blocks=1,
                         mode="MOL")
    m = WaveRNN(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, 760).items()})
    mel = torch.from_numpy(syn.make_mel(d.feat_dims, 40, 761))[None]
    out = m.generate(mel, None, False, 11000, 550, False, seed=3, verbose=False)
    assert out.shape[0] == (40 - 1) * d.hop_length and np.isfinite(out).all() and np.abs(out).max() <= 1.0


@pytest.mark.parametrize("bits,B", [(10, 1), (10, 3), (11, 2)])
def test_raw_more_than_512_classes(bits, B, monkeypatch):
    """bits 10 / 11 (1 024 / 2 048 classes): the sampler's generic form (raw_sample_any), labels
    bit-exact vs the oracle."""
    from oracle import oracle
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.FatchordDims(bits=bits, mode="RAW")
    state = syn.make_fatchord_state(d, 770 + bits)
    mels, aux = syn.make_conditioning(B, 150, d.feat_dims, d.res_out_dims, 771 + B)
    noise = syn.make_noise("RAW", B, 150, d.n_classes, 772 + B)
    _, ref_lab = oracle.fatchord_loop(state, "RAW", mels, aux, noise)
    loop = _loop(d)
    loop.set_weights(state)
    _, lab = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=True)
    np.testing.assert_array_equal(lab.cpu().numpy(), ref_lab)


def test_deepmind_quantisation_512():
    """deepmind quantisation 512 (the rows kernel's generic sampler): labels bit-exact vs the oracle."""
    from oracle import oracle
    from wavernn_amd.loop import DeepmindLoop
    d = syn.DeepmindDims(hidden_size=128, quantisation=512)
    B, L = 3, 150
    state = syn.make_deepmind_state(d, 780)
    noise = syn.make_dm_noise(B, L, d.quantisation, 781)
    _, _, ref = oracle.deepmind_loop(state, B, L, noise)
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(state)
    _, comb = loop.generate(B, L, noise=torch.from_numpy(noise).to(DEV))
    np.testing.assert_array_equal(comb.cpu().numpy().astype(np.int64), ref)
