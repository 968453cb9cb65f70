"""Config 4's production route against the reference itself.

BASELINE config 4 is the rnn-896 model with its GRU matrices pruned to 95 % in 4x4 blocks, 8
utterances per GPU.  bench.py times it through `sharding.generate_sharded` → `generate_many`: the
MelResNet kernel, the conditioning terms at frame rate at rnn 896 (frame_terms.hip), ONE launch
of `fatchord_xcds_kernel` with the 8 utterances as its rows (one per XCD), the float64 post.
The fixtures were written by running the reference's own `generate()`
(/root/reference/models/fatchord_version.py:169-264) on the pre-masked dense weights with
injected sampler draws (tests/golden/make_golden.py):
  * gen_sparse896_5s_unbatched — one 5 s utterance (T = 401, 110 275 steps) through generate();
  * gen_sparse896_8utt         — 8 utterances (T = 41, mel seeds 60..67) vocoded one by one, as
                                 gen_wavernn.py:11-35 does; utterance i took draws noise[:, i].
Here the drop-in runs its DEFAULT entry (no WRNN_* override) and the kernel it picked is checked
(path 6 = fatchord_xcds_kernel).  MoL tolerance |Δ| <= MOL_TOL = 1e-5 per sample,
the first index over it reported."""
import os

import numpy as np
import pytest
import torch

from tests.golden import fixtures as gf

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
OVERRIDES = ("WRNN_PATH", "WRNN_NO_FRAME_TERMS", "WRNN_TORCH_MELRESNET", "WRNN_SPARSE")


def _first_over(diff: np.ndarray, tol: float) -> str:
    bad = np.argwhere(diff > tol)
    if not len(bad):
        return "none"
    i = tuple(int(v) for v in bad[0])
    return f"first at {i} (|Δ| {diff[i]:.3g}), {len(bad)} of {diff.size} over"


def _no_overrides():
    for k in OVERRIDES:
        assert k not in os.environ, f"{k} set: this test pins the DEFAULT entry"


def _model(d, state):
    from wavernn_amd.fatchord_version import WaveRNN
    m = WaveRNN(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
    return m


def _check(got, ref, what):
    diff = np.abs(got - ref)
    assert diff.max() <= gf.MOL_TOL, f"{what}: max |Δ| {diff.max():.3g}, {_first_over(diff, gf.MOL_TOL)}"
    print(f"{what}: max |Δ| {diff.max():.3g} (mean {diff.mean():.3g}) over {diff.size} samples")


@pytest.mark.parametrize("name", gf.GEN_SPARSE_CASES)
def test_sparse896_generate_vs_reference(name):
    _no_overrides()
    fx = gf.load(name)
    d, state, mel, noise = gf.gen_inputs(fx)
    m = _model(d, state)
    mel_t = torch.from_numpy(mel)[None]
    out = m.generate(mel_t, None, False, int(fx["target"]), int(fx["overlap"]), bool(fx["mu_law"]),
                     noise=noise, verbose=False)
    h = m.loop_handle()
    assert h.info["last_path"] == 6 and h.info["sparse_blocks"] > 0, h.info
    assert out.dtype == np.float64 and out.shape == (int(fx["out_len"]),)
    s = int(fx["out_stride"])
    _check(out[::s], fx["output"], f"{name} output")
    assert abs(out.sum() - float(fx["out_sum"])) <= gf.MOL_TOL * out.size
    # per-step loop outputs of the same entry against the reference's sampler outputs
    mel_f, aux, _ = m.frames(mel_t)
    y, _ = h.generate_frames(m._upsample_spec(), mel_f, aux, 0, int(fx["overlap"]),
                             noise=torch.from_numpy(noise).to(DEV))
    _check(y.cpu().numpy(), fx["raw"], f"{name} loop outputs")


@pytest.mark.parametrize("name", gf.GEN_MANY_CASES)
def test_sparse896_generate_many_one_launch_vs_reference(name):
    """The 8 utterances as the rows of ONE launch (generate_many, the bench's config-4 call),
    noise in the launch's row order, against the reference's one-by-one outputs."""
    _no_overrides()
    fx = gf.load(name)
    d, state, mels, noise = gf.gen_many_inputs(fx)
    m = _model(d, state)
    ms = [torch.from_numpy(x)[None] for x in mels]
    outs = m.generate_many(ms, None, False, int(fx["target"]), int(fx["overlap"]), bool(fx["mu_law"]), noise=noise)
    h = m.loop_handle()
    assert h.info["last_path"] == 6 and h.info["sparse_blocks"] > 0, h.info
    s = int(fx["out_stride"])
    assert len(outs) == len(mels)
    for i, o in enumerate(outs):
        assert o.dtype == np.float64 and o.shape == (int(fx["out_len"]),)
        _check(o[::s], fx["output"][i], f"utterance {i} output")
        assert abs(o.sum() - float(fx["out_sum"][i])) <= gf.MOL_TOL * o.size
    mel_f, aux, _ = m.frames(torch.cat(ms, 0))
    y, _ = h.generate_frames(m._upsample_spec(), mel_f, aux, 0, int(fx["overlap"]),
                             noise=torch.from_numpy(noise).to(DEV))
    assert y.shape == fx["raw"].shape
    _check(y.cpu().numpy(), fx["raw"], "8-row launch loop outputs")


@pytest.mark.parametrize("name", gf.GEN_MANY_CASES)
def test_sparse896_sharded_leg_vs_reference(name):
    """The sharded entry bench.py calls (sharding.generate_sharded over the 8 mels; world 1 on
    this one-GPU box), with the reference's draws injected through its `noise` argument."""
    _no_overrides()
    from wavernn_amd import sharding
    fx = gf.load(name)
    d, state, mels, noise = gf.gen_many_inputs(fx)
    m = _model(d, state)
    ms = [torch.from_numpy(x)[None] for x in mels]
    outs = sharding.generate_sharded(m, ms, batched=False, target=int(fx["target"]), overlap=int(fx["overlap"]),
                                     mu_law=bool(fx["mu_law"]), noise=noise)
    s = int(fx["out_stride"])
    for i, o in enumerate(outs):
        _check(np.asarray(o)[::s], fx["output"][i], f"sharded utterance {i}")
