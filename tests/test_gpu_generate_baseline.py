"""The SHIPPED generate() entry at BASELINE sizes against the reference itself.

The fixtures (tests/golden/make_golden.py, `gen_*` BASELINE cases) were written by running the
reference's own `WaveRNN.generate()` (/root/reference/models/fatchord_version.py:169-264) on the
CPU with injected sampler draws.  Here the drop-in `generate()` runs with the same weights, mel and
draws and its DEFAULT entry — no WRNN_PATH / WRNN_NO_FRAME_TERMS / WRNN_TORCH_MELRESNET override:
the fused MelResNet kernel (wrnn_melresnet), `wrnn_generate_frames` (conditioning terms formed at
frame rate) and the persistent loop kernel the C-ABI picks for the row count, then the float64
post-processing kernel.  These are the code paths bench.py times:
  * gen_raw_1s_unbatched  — config 1 exactly (RAW 9-bit, 1 s, 22 275 steps);
  * gen_mol_5s_unbatched  — config 2, the headline (110 275 steps, fatchord_xcd_kernel);
  * gen_mol_5s_batched    — the same utterance in the reference's default fold-batched mode
                            (hparams.py:58-60: 10 folds x 12 100 steps, fatchord_xcdm_kernel);
  * gen_mol_60s_batched   — config 3 (115 folds x 12 100 steps).
Tolerances: RAW — labels bit-exact, so the float64 output equals the reference's
up to the device pow/sqrt rounding (rtol 1e-12); MoL — |Δ| <= MOL_TOL = 1e-5 per sample, over the
stored output samples and the stored per-step loop outputs; the first index over tolerance is
reported.  Under MoL feedback a divergence at one step would change every later sample of its
row, so the strided fixtures of the long cases still see it."""
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


@pytest.fixture(scope="module")
def models():
    return {}


def _model(fx, models):
    from wavernn_amd.fatchord_version import WaveRNN
    d, state, mel, noise = gf.gen_inputs(fx)
    key = str(fx["dims"])
    if key not in models:
        m = WaveRNN(**d.ctor_kwargs()).to(DEV)
        m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
        models[key] = m
    return d, models[key], mel, noise


@pytest.mark.parametrize("name", gf.GEN_BASELINE_CASES)
def test_dropin_generate_at_baseline_size(name, models):
    for k in OVERRIDES:
        assert k not in os.environ, f"{k} set: this test pins the DEFAULT entry"
    fx = gf.load(name)
    d, m, mel, noise = _model(fx, models)
    batched, target, overlap = bool(fx["batched"]), int(fx["target"]), int(fx["overlap"])
    mel_t = torch.from_numpy(mel)[None]
    out = m.generate(mel_t, None, batched, target, overlap, bool(fx["mu_law"]), noise=noise, verbose=False)
    assert out.dtype == np.float64 and out.shape == (int(fx["out_len"]),)
    # which kernel the default entry picked (what bench.py times for this shape)
    path = m.loop_handle().info["last_path"]
    expect = {"gen_raw_1s_unbatched": 7, "gen_mol_5s_unbatched": 5, "gen_mol_5s_batched": 7,
              "gen_mol_60s_batched": 7}[name]
    assert path == expect, f"default entry ran path {path}, expected {expect}"
    s = int(fx["out_stride"])
    got, ref = out[::s], fx["output"]
    assert got.shape == ref.shape
    if d.mode == "RAW":
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-300)
    else:
        diff = np.abs(got - ref)
        assert diff.max() <= gf.MOL_TOL, f"output: max |Δ| {diff.max():.3g}, {_first_over(diff, gf.MOL_TOL)}"
        assert abs(out.sum() - float(fx["out_sum"])) <= gf.MOL_TOL * out.size
        print(f"{name}: output max |Δ| {diff.max():.3g} (mean {diff.mean():.3g}) over {diff.size} samples")

    # the loop outputs of the same entry (frames -> wrnn_generate_frames), per step, vs the
    # reference's per-step sampler outputs
    mel_f, aux, _ = m.frames(mel_t)
    nz = torch.from_numpy(noise).to(DEV)
    y, lab = m.loop_handle().generate_frames(m._upsample_spec(), mel_f, aux, target if batched else 0, overlap,
                                             noise=nz, want_labels=d.mode == "RAW")
    rows = fx["raw_rows"] if "raw_rows" in fx else np.arange(y.shape[0])
    if d.mode == "RAW":
        lab = lab.cpu().numpy()
        eq = lab[rows] == fx["raw"].astype(np.int32)
        assert eq.all(), f"RAW labels: {eq.mean():.6f} equal, first mismatch {tuple(np.argwhere(~eq)[0])}"
        print(f"{name}: {eq.size} labels bit-exact; output max rel |Δ| "
              f"{np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)):.3g}")
    else:
        y = y.cpu().numpy()
        diff = np.abs(y[rows] - fx["raw"])
        assert diff.max() <= gf.MOL_TOL, f"loop outputs: max |Δ| {diff.max():.3g}, {_first_over(diff, gf.MOL_TOL)}"
        print(f"{name}: loop outputs of rows {list(rows)[:4]}{'…' if len(rows) > 4 else ''} max |Δ| {diff.max():.3g} "
              f"over {diff.size} row-steps")
        if "raw_strided" in fx:
            st = int(fx["raw_stride"])
            diff = np.abs(y[:, ::st] - fx["raw_strided"])
            assert diff.max() <= gf.MOL_TOL, f"strided rows: {_first_over(diff, gf.MOL_TOL)}"
