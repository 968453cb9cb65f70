"""The RAW (9-bit softmax) head of the XCD-resident many-row kernel (csrc/fatchord_xcdm.hip,
kRaw: fc3 as a twelfth MFMA set with its A operands in LDS, f2 and the logits as hop vectors,
softmax → Categorical ≡ argmax(p / q) sampled per row; fatchord_version.py:231-237) through the
C-ABI: the default RAW rnn-512 path at every row count (wrnn_info.last_path 7).

Labels are bit-exact against the reference fixtures and the oracle under injected Exp(1) draws
(SURVEY.md §8(c)); the samples are label_to_x of the labels."""
import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
XCDM = 7


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


def _loop(d=syn.DEFAULT_RAW):
    from wavernn_amd.loop import FatchordLoop
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes, device=0)
    if loop.info["xcdm_rows"] == 0:
        pytest.skip("many-row XCD kernel unavailable on this device")
    return loop


def _check(out, lab, ref, ref_lab):
    lab = lab.cpu().numpy()
    eq = lab == ref_lab
    assert eq.all(), f"{eq.mean():.6f} of the labels equal, first mismatch (row, step) {np.argwhere(~eq)[0].tolist()}"
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("name", ["loop_raw_b1", "loop_raw_b3", "loop_raw_1s"])
def test_raw_xcdm_vs_reference_fixture(name, monkeypatch):
    """Fixtures made by running the reference (loop_raw_1s: a full 1 s, 22 275 steps)."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    fx = gf.load(name)
    d, state, mels, aux, noise = gf.loop_inputs(fx)
    loop = _loop(d)
    loop.set_weights(state)
    out, lab = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=True)
    assert loop.info["last_path"] == XCDM, loop.info
    labels = fx["labels"].astype(np.int32)
    x = (2.0 * labels.astype(np.float32)) / np.float32(d.n_classes - 1.0) - np.float32(1.0)
    _check(out, lab, x.astype(np.float32), labels)


@pytest.mark.parametrize("B", [2, 8, 10, 33, 57, 80, 128])
def test_raw_xcdm_vs_oracle(B, monkeypatch):
    """One quad per XCD (B <= 32: every workgroup samples every row), the two-level sampler and
    the 16x16x4 form (B > 32), ragged XCDs."""
    from oracle import oracle
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.DEFAULT_RAW
    L = 160
    state = syn.make_fatchord_state(d, 800 + B)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 801 + B)
    noise = syn.make_noise("RAW", B, L, d.n_classes, 802 + B)
    ref, ref_lab = oracle.fatchord_loop(state, "RAW", mels, aux, noise)
    loop = _loop()
    loop.set_weights(state)
    out, lab = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=True)
    assert loop.info["last_path"] == XCDM, loop.info
    _check(out, lab, ref, ref_lab)


@pytest.mark.parametrize("B", [3, 40])
def test_raw_xcdm_time_chunks(B, monkeypatch):
    """Launches split in time carry the recurrent state: the oracle's labels, and the labels of a
    single launch under Philox (the draws pre-filled per chunk, keyed like every other kernel)."""
    from oracle import oracle
    d = syn.DEFAULT_RAW
    L = 300
    state = syn.make_fatchord_state(d, 820 + B)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 821 + B)
    noise = syn.make_noise("RAW", B, L, d.n_classes, 822 + B)
    ref, ref_lab = oracle.fatchord_loop(state, "RAW", mels, aux, noise)
    loop = _loop()
    loop.set_weights(state)
    cond = _cond(mels, aux)
    _, whole = loop.generate(cond, seed=5, want_labels=True)
    monkeypatch.setenv("WRNN_TERMS_MB", "3")
    out, lab = loop.generate(cond, noise=torch.from_numpy(noise).to(DEV), want_labels=True)
    assert loop.info["last_path"] == XCDM
    _check(out, lab, ref, ref_lab)
    _, chunked = loop.generate(cond, seed=5, want_labels=True)
    assert torch.equal(chunked, whole)


def test_raw_xcdm_more_rows_than_one_launch(monkeypatch):
    """130 rows: a 128-row launch and a 2-row one."""
    from oracle import oracle
    monkeypatch.delenv("WRNN_PATH", raising=False)
    d = syn.DEFAULT_RAW
    B, L = 130, 80
    state = syn.make_fatchord_state(d, 840)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 841)
    noise = syn.make_noise("RAW", B, L, d.n_classes, 842)
    ref, ref_lab = oracle.fatchord_loop(state, "RAW", mels, aux, noise)
    loop = _loop()
    loop.set_weights(state)
    out, lab = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=True)
    _check(out, lab, ref, ref_lab)


@pytest.mark.parametrize("B", [1, 12])
def test_raw_xcdm_agrees_with_rows_kernel_under_philox(B, monkeypatch):
    """Philox draws keyed by (seed, row_offset + b, step, k): the same labels from the many-row
    XCD kernel and the multi-row kernel, including a row offset."""
    d = syn.DEFAULT_RAW
    L = 200
    state = syn.make_fatchord_state(d, 860)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 861)
    cond = _cond(mels, aux)
    res = {}
    for p, path in (("", XCDM), ("rows", 2)):
        monkeypatch.setenv("WRNN_PATH", p)
        loop = _loop()
        loop.set_weights(state)
        res[p] = loop.generate(cond, seed=9, row_offset=4, want_labels=True)[1]
        assert loop.info["last_path"] == path
        loop.close()
    assert torch.equal(res[""], res["rows"])
