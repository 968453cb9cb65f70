"""The in-kernel Philox stream (noise == NULL) against its numpy restatement.

Every throughput number runs the loop kernels with noise == NULL: the sampler draws come from
Philox-4x32-10 inside the kernels (`philox_noise`, csrc/wrnn_device.h) or from the fill kernel
ahead of them.  Before this file only kernel-vs-kernel agreement pinned that stream.  Here:
  1. the device draws (C-ABI wrnn_philox_draws) against oracle/philox.py — itself pinned to the
     published known-answer vectors (tests/test_philox.py): MoL uniforms bit-exact; the Exp(1)
     draws within the bound below (the device's fp32 logf vs float64 log rounded once);
  2. each kernel family run twice — noise=None with (seed, row_offset), then with the
     HOST-restated draws injected — RAW and deepmind labels bit-exact, MoL within MOL_TOL
     (observed: identical).  The injected-noise route of every kernel is what the reference
     fixtures pin (tests/test_gpu_parity.py, test_gpu_generate_baseline.py), so this closes the
     chain from the bench's audio to the reference: the draw distributions are those of
     utils/distribution.py:106,118, fatchord_version.py:232-235, deepmind_version.py:130,150.
The keying covers rows past 2^32, 64-bit seeds, and time-chunked launches (fill offsets)."""
import numpy as np
import pytest
import torch

from oracle import philox as ph
from tests.golden import fixtures as gf
from wavernn_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
BIG_SEED = (0xDEADBEEF << 32) | 0x12345678


def _exp_close(got: np.ndarray, ref: np.ndarray, what: str):
    """Device -log(u) (float64 log, one rounding) vs numpy's: bit-equal but for the rare draw
    whose float64 logs differ in their last bit across a float32 rounding boundary (~2^-29 per
    draw): at most one fp32 ulp, on at most 1e-5 of the draws, with no bias."""
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    exact = float((got == ref).mean())
    print(f"{what}: {exact:.6f} of {got.size} draws bit-equal, max {np.max(d / ulp):.2f} ulp")
    assert (d <= ulp).all(), f"{what}: first draw over 1 ulp at {tuple(np.argwhere(d > ulp)[0])}"
    assert exact >= 1 - 1e-5, what


@pytest.mark.parametrize("mode,K", [("MOL", 11), ("RAW", 512), ("DM", 512), ("RAW", 7)])
@pytest.mark.parametrize("seed,row0,step0", [(1234, 0, 0), (BIG_SEED, (1 << 32) - 3, 70000)])
def test_device_draws_vs_restatement(mode, K, seed, row0, step0):
    from wavernn_amd.loop import philox_draws
    rows, steps = 6, 300
    got = philox_draws(seed, row0, rows, steps, K, mode, step0=step0).cpu().numpy()
    ref = ph.philox_draws(seed, row0, rows, step0, steps, K, mol=mode == "MOL")
    assert got.shape == ref.shape == (steps, rows, K)
    if mode == "MOL":
        eq = got == ref
        assert eq.all(), f"{eq.mean():.6f} equal, first mismatch {tuple(np.argwhere(~eq)[0])}"
    else:
        _exp_close(got, ref, f"{mode} K={K}")


def test_device_draws_reject_bad_arguments():
    from wavernn_amd import _native as nat
    from wavernn_amd.loop import philox_draws
    with pytest.raises(nat.WrnnError):
        philox_draws(1, 0, 0, 10, 11, "MOL")


def _fatchord_loop(d, state):
    from wavernn_amd.loop import FatchordLoop
    lp = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    lp.set_weights(state)
    return lp


def _cond(mels, aux):
    return torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(DEV)


# (kernel forced by WRNN_PATH or "" for the default pick, dims, prune, rows, steps, expected path)
FAMILIES = [
    ("xcd", "", syn.DEFAULT_MOL, 0.0, 3, 500, 5),             # the headline's kernel
    ("xcdm-mol", "", syn.DEFAULT_MOL, 0.0, 12, 300, 7),       # fold-batched / config 3
    ("xcdm-raw", "", syn.DEFAULT_RAW, 0.0, 3, 400, 7),        # RAW at every row count (fill kernel)
    ("xcds", "", syn.SPARSE896_MOL, 0.95, 2, 300, 6),         # config 4
    ("rows-mol", "rows", syn.DEFAULT_MOL, 0.0, 2, 200, 2),
    ("rows-raw", "rows", syn.DEFAULT_RAW, 0.0, 2, 200, 2),
    ("latency", "latency", syn.DEFAULT_MOL, 0.0, 1, 200, 1),
    ("split", "split", syn.DEFAULT_MOL, 0.0, 1, 200, 4),
]


@pytest.mark.parametrize("name,force,d,prune,B,L,want_path", FAMILIES, ids=[f[0] for f in FAMILIES])
def test_kernel_in_kernel_draws_equal_restated_injection(name, force, d, prune, B, L, want_path, monkeypatch):
    if force:
        monkeypatch.setenv("WRNN_PATH", force)
    else:
        monkeypatch.delenv("WRNN_PATH", raising=False)
    state = syn.make_fatchord_state(d, 40)
    if prune:
        from wavernn_amd.pruning import prune_state
        state = prune_state(state, prune)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 41)
    cond = _cond(mels, aux)
    loop = _fatchord_loop(d, state)
    seed, r0 = BIG_SEED + B, 5 + (1 << 32)
    y0, lab0 = loop.generate(cond, seed=seed, row_offset=r0, want_labels=True)
    assert loop.info["last_path"] == want_path, loop.info
    noise = ph.philox_draws(seed, r0, B, 0, L, 11 if d.mode == "MOL" else d.n_classes, mol=d.mode == "MOL")
    y1, lab1 = loop.generate(cond, noise=torch.from_numpy(noise).to(DEV), want_labels=True)
    assert loop.info["last_path"] == want_path
    if d.mode == "RAW":
        a, b = lab0.cpu().numpy(), lab1.cpu().numpy()
        eq = a == b
        assert eq.all(), f"{name}: {eq.mean():.6f} labels equal, first mismatch {tuple(np.argwhere(~eq)[0])}"
        assert len(np.unique(a)) > 20
        print(f"{name}: {a.size} labels bit-exact")
    else:
        diff = (y0 - y1).abs().max().item()
        print(f"{name}: max |Δ| {diff:.3g} ({'identical' if diff == 0 else 'within tolerance'})")
        # the same draws through the same arithmetic: bit-identical (round 6: observed on every family)
        assert torch.equal(y0, y1), diff
    loop.close()


def test_xcdm_raw_time_chunks_keyed_by_global_step(monkeypatch):
    """RAW through the many-row kernel in several time chunks (each chunk's draws filled at its
    step offset): still the restated stream."""
    monkeypatch.delenv("WRNN_PATH", raising=False)
    monkeypatch.setenv("WRNN_TERMS_MB", "1")
    d = syn.DEFAULT_RAW
    B, L = 2, 900
    state = syn.make_fatchord_state(d, 42)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 43)
    loop = _fatchord_loop(d, state)
    _, lab0 = loop.generate(_cond(mels, aux), seed=77, row_offset=3, want_labels=True)
    noise = ph.philox_draws(77, 3, B, 0, L, d.n_classes, mol=False)
    _, lab1 = loop.generate(_cond(mels, aux), noise=torch.from_numpy(noise).to(DEV), want_labels=True)
    assert torch.equal(lab0, lab1)


@pytest.mark.parametrize("force,B,L,noise_mb,want_path", [("", 8, 400, None, 8), ("", 5, 600, "1", 8),
                                                          ("rows", 3, 200, None, 3)])
def test_deepmind_in_kernel_draws_equal_restated_injection(force, B, L, noise_mb, want_path, monkeypatch):
    """deepmind: XCD-resident kernel (fill kernel; noise_mb=1 forces several fills at step
    offsets) and the rows kernel (in-kernel draws): coarse and fine labels bit-exact."""
    from wavernn_amd.loop import DeepmindLoop
    if force:
        monkeypatch.setenv("WRNN_PATH", force)
    else:
        monkeypatch.delenv("WRNN_PATH", raising=False)
    if noise_mb:
        monkeypatch.setenv("WRNN_DM_NOISE_MB", noise_mb)
    d = syn.DEFAULT_DM
    loop = DeepmindLoop(d.hidden_size, d.quantisation)
    loop.set_weights(syn.make_deepmind_state(d, 44))
    seed, r0 = BIG_SEED, (1 << 32) + 11
    _, c0 = loop.generate(B, L, seed=seed, row_offset=r0)
    assert loop.info["last_path"] == want_path
    noise = ph.philox_draws(seed, r0, B, 0, L, 2 * d.quantisation, mol=False)
    _, c1 = loop.generate(B, L, noise=torch.from_numpy(noise).to(DEV))
    a, b = c0.cpu().numpy(), c1.cpu().numpy()
    eq = a == b
    assert eq.all(), f"{eq.mean():.6f} equal, first mismatch {tuple(np.argwhere(~eq)[0])}"
    assert len(np.unique(a)) > 50
    loop.close()


def test_dropin_generate_philox_equals_restated_noise():
    """The bench's call: the drop-in generate() of the headline model with seed= (noise None)
    equals the same call with the restated draws injected — so the bench's audio is the audio
    the reference fixtures pin under injection."""
    from wavernn_amd.fatchord_version import WaveRNN
    d = syn.DEFAULT_MOL
    m = WaveRNN(**d.ctor_kwargs()).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, 45).items()})
    mel = torch.from_numpy(syn.make_mel(d.feat_dims, 30, 46))[None]
    a = m.generate(mel, None, False, 11000, 550, True, seed=2718, verbose=False)
    L = 30 * d.hop_length                                  # loop steps of a 30-frame mel (unbatched)
    b_noise = ph.philox_draws(2718, 0, 1, 0, L, 11, mol=True)
    b = m.generate(mel, None, False, 11000, 550, True, noise=b_noise, verbose=False)
    assert m.loop_handle().info["last_path"] == 5
    err = np.abs(a - b).max()
    print(f"drop-in generate: Philox vs restated injection max |Δ| {err:.3g}")
    assert err <= gf.MOL_TOL
