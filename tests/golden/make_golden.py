"""Generate the golden fixtures by running the REFERENCE `WaveRNN.generate()` on CPU.

Dev tool: runs only in the build container, where the read-only reference lives at
/root/reference.  The reference never travels; only the `.npz` data it produced does.

    PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_golden.py [case ...]

How the reference is made importable, all in-memory, nothing written
to /root/reference:
  * `sys.modules['librosa']` = stub whose `output.write_wav` is a no-op (only
    `utils/dsp.py:22-23` save_wav touches librosa on this path);
  * `np.cumproduct = np.cumprod` (removed in numpy 2; used at fatchord_version.py:68).

Noise injection (so the fixtures are a pure-arithmetic contract, SURVEY.md §8(b,c)):
  * MOL: `torch.Tensor.uniform_` is intercepted only while the reference's own
    `sample_from_discretized_mix_logistic` (utils/distribution.py:87-123) runs; the two
    draws per step (u1 (1,B,10) at :106, u2 (1,B) at :118) are served from our noise.
  * RAW: `torch.distributions.Categorical.sample` is replaced by argmax(probs / q) with
    our q ~ Exp(1) — the exact fast path torch.multinomial(n=1) takes; this script
    re-verifies that equivalence against torch's own sampler before using it.
  * deepmind (dm_*): `models.deepmind_version.stream` (progress printer, crashes with the
    reference's own arguments at :159) is replaced by a no-op; the two Categorical.sample
    calls per step (coarse :130, fine :150) are served q_coarse then q_fine.
Inputs come from `wavernn_amd.synthetic` (seeded numpy); each fixture stores the
SHA-256 of its inputs so the tests can prove they regenerate the same inputs.
"""
from __future__ import annotations

import os
import sys
import time
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wavernn_amd import synthetic as syn  # noqa: E402


def import_reference():
    if REF not in sys.path:
        sys.path.insert(1, REF)
    np.cumproduct = np.cumprod
    lib = types.ModuleType("librosa")
    lib.output = types.SimpleNamespace(write_wav=lambda *a, **k: None)
    sys.modules["librosa"] = lib
    from utils import hparams as hp  # noqa
    if not hp.is_configured():
        hp.configure(os.path.join(REF, "hparams.py"))
    import models.fatchord_version as fv  # noqa
    return fv


def check_categorical_equivalence(n: int = 64):
    """torch Categorical(p).sample() == argmax(p/q), q = exponential_ from the same RNG state."""
    for s in range(n):
        logits = torch.randn(3, 512) * 3
        p = torch.softmax(logits, 1)
        torch.manual_seed(s)
        a = torch.distributions.Categorical(p).sample()
        torch.manual_seed(s)
        probs = p / p.sum(-1, keepdim=True)
        q = torch.empty_like(probs).exponential_(1)
        b = (probs / q).argmax(-1)
        assert torch.equal(a, b), "Categorical fast-path equivalence broken"


class NoiseInjector:
    """Serve per-step noise [L][B][K] to the reference sampler and record its outputs."""

    def __init__(self, fv, mode: str, noise: np.ndarray):
        self.fv, self.mode, self.noise = fv, mode, noise
        self.t = 0
        self.draw = 0
        self.active = False
        self.samples = []   # MOL: (B,) float32 per step ; RAW: (B,) int64 labels per step
        self._saved = {}

    def __enter__(self):
        fv, inj = self.fv, self
        if self.mode == "MOL":
            orig_sampler = fv.sample_from_discretized_mix_logistic
            orig_uniform = torch.Tensor.uniform_

            def uniform_hook(tensor, a=0.0, b=1.0, *args, **kw):
                if not inj.active:
                    return orig_uniform(tensor, a, b, *args, **kw)
                step = inj.noise[inj.t]                     # (B, 11)
                if inj.draw == 0:
                    assert tuple(tensor.shape) == (1, step.shape[0], 10), tensor.shape
                    tensor.copy_(torch.from_numpy(step[None, :, :10]))
                else:
                    assert tuple(tensor.shape) == (1, step.shape[0]), tensor.shape
                    tensor.copy_(torch.from_numpy(step[None, :, 10]))
                inj.draw += 1
                return tensor

            def sampler(y, *a, **k):
                inj.active, inj.draw = True, 0
                try:
                    x = orig_sampler(y, *a, **k)
                finally:
                    inj.active = False
                assert inj.draw == 2
                inj.samples.append(x.reshape(-1).detach().numpy().astype(np.float32).copy())
                inj.t += 1
                return x

            self._saved = dict(sampler=orig_sampler, uniform=orig_uniform)
            fv.sample_from_discretized_mix_logistic = sampler
            torch.Tensor.uniform_ = uniform_hook
        else:
            orig_sample = torch.distributions.Categorical.sample

            def cat_sample(dist, sample_shape=torch.Size()):
                q = torch.from_numpy(inj.noise[inj.t])    # (B, n_classes)
                lab = (dist.probs / q).argmax(-1)
                inj.samples.append(lab.numpy().astype(np.int64).copy())
                inj.t += 1
                return lab

            self._saved = dict(sample=orig_sample)
            torch.distributions.Categorical.sample = cat_sample
        return self

    def __exit__(self, *exc):
        if self.mode == "MOL":
            self.fv.sample_from_discretized_mix_logistic = self._saved["sampler"]
            torch.Tensor.uniform_ = self._saved["uniform"]
        else:
            torch.distributions.Categorical.sample = self._saved["sample"]
        return False


def build_ref_model(fv, d: syn.FatchordDims, state):
    m = fv.WaveRNN(**d.ctor_kwargs())
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
    return m


def fold_count(L: int, target: int, overlap: int) -> int:
    """Reference fold_with_overlap (fatchord_version.py:322-330)."""
    n = (L - overlap) // (target + overlap)
    if L - (n * (overlap + target) + overlap) != 0:
        n += 1
    return n


# ----------------------------------------------------------------------------- loop cases
def loop_case(fv, name, d: syn.FatchordDims, B: int, L: int, wseed=0, cseed=2, nseed=3, prune=0.0):
    """Drive the reference loop (fatchord_version.py:201-241) on given folded conditioning.
    prune > 0: GRU weights block-pruned to that sparsity first (wavernn_amd/pruning.py)."""
    state = syn.make_fatchord_state(d, wseed)
    if prune > 0:
        from wavernn_amd.pruning import prune_state
        state = prune_state(state, prune)
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, cseed)
    noise = syn.make_noise(d.mode, B, L, d.n_classes, nseed)
    model = build_ref_model(fv, d, state)
    # upsample/fold are bypassed: the loop consumes our conditioning verbatim.
    if B == 1:   # unbatched: generate() loops directly on the upsample output
        up = torch.from_numpy(mels), torch.from_numpy(aux)
    else:        # batched: fold_with_overlap hands our [B][L][·] conditioning to the loop
        up = torch.zeros(1, L, d.feat_dims), torch.zeros(1, L, d.res_out_dims)
    model.upsample.forward = lambda m: up
    seq = iter([torch.from_numpy(mels), torch.from_numpy(aux)])
    model.fold_with_overlap = lambda x, target, overlap: next(seq)
    mel_in = torch.zeros(1, d.feat_dims, 30)
    t0 = time.time()
    with NoiseInjector(fv, d.mode, noise) as inj:
        try:
            model.generate(mel_in, "/dev/null", batched=(B > 1), target=L - 2 * 100,
                           overlap=100, mu_law=True)
        except Exception:
            # post-processing after the loop may reject these synthetic lengths; the
            # per-step outputs we need were recorded by the hooks.
            pass
    dt = time.time() - t0
    assert inj.t == L, (inj.t, L)
    outs = np.stack(inj.samples)  # [L][B]
    rec = dict(kind="loop", mode=d.mode, B=B, L=L, wseed=wseed, cseed=cseed, nseed=nseed, prune=prune,
               dims=np.array(repr(d)), ref_seconds=dt,
               state_sha=syn.state_digest(state), cond_sha=syn.digest(mels, aux),
               noise_sha=syn.digest(noise))
    if d.mode == "RAW":
        rec["labels"] = outs.T.astype(np.int16)           # [B][L]
    else:
        rec["samples"] = outs.T.astype(np.float32)        # [B][L]
    return rec


# ------------------------------------------------------------------------- deepmind cases
def dm_case(fv, name, d: syn.DeepmindDims, L: int, wseed=0, nseed=3):
    """deepmind_version.WaveRNN.generate(seq_len) (:75-165), batch 1, injected Exp(1) noise."""
    import models.deepmind_version as dm
    dm.stream = lambda *a, **k: None
    state = syn.make_deepmind_state(d, wseed)
    noise = syn.make_dm_noise(1, L, d.quantisation, nseed)           # [L][1][2Q]
    Q = d.quantisation
    draws = noise.reshape(L, 1, 2, Q).transpose(0, 2, 1, 3).reshape(2 * L, 1, Q)   # coarse, fine, …
    m = dm.WaveRNN(**d.ctor_kwargs())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()}, strict=True)
    orig = torch.distributions.Categorical.sample
    calls = [0]

    def cat_sample(dist, sample_shape=torch.Size()):
        q = torch.from_numpy(draws[calls[0]])
        calls[0] += 1
        return (dist.probs / q).argmax(-1)

    torch.distributions.Categorical.sample = cat_sample
    t0 = time.time()
    try:
        output, coarse, fine = m.generate(L)
    finally:
        torch.distributions.Categorical.sample = orig
    dt = time.time() - t0
    assert calls[0] == 2 * L
    return dict(kind="dm", L=L, wseed=wseed, nseed=nseed, dims=np.array(repr(d)), ref_seconds=dt,
                state_sha=syn.state_digest(state), noise_sha=syn.digest(noise),
                coarse=np.asarray(coarse).astype(np.int16).reshape(1, L),
                fine=np.asarray(fine).astype(np.int16).reshape(1, L),
                output=np.asarray(output).astype(np.int32).reshape(1, L))


# ------------------------------------------------------------------------------ e2e cases
def gen_case(fv, name, d: syn.FatchordDims, T: int, batched: bool, target: int, overlap: int,
             mu_law: bool, wseed=0, mseed=1, nseed=3, cond_stride=25, out_stride=1,
             raw_rows=None, raw_stride=0, prune=0.0):
    """Full reference generate(): pad → upsample → fold → loop → unfold/mu-law/fade.

    BASELINE-size cases keep the fixture small: `out_stride` stores every k-th output sample
    (float64), `raw_rows` keeps the per-step loop outputs of those fold rows only, and
    `raw_stride` > 0 additionally keeps every row at every raw_stride-th step.  Under MoL
    feedback a divergence at one step changes every later sample of its row, so a strided
    view still catches it.  prune > 0: the GRU weights block-pruned to that sparsity first
    (config 4's model, wavernn_amd/pruning.py); the reference runs the pre-masked dense weights."""
    state = syn.make_fatchord_state(d, wseed)
    if prune > 0:
        from wavernn_amd.pruning import prune_state
        state = prune_state(state, prune)
    mel = syn.make_mel(d.feat_dims, T, mseed)
    L = d.hop_length * T
    B = fold_count(L, target, overlap) if batched else 1
    Lf = target + 2 * overlap if batched else L
    noise = syn.make_noise(d.mode, B, Lf, d.n_classes, nseed)
    model = build_ref_model(fv, d, state)
    captured = {}
    orig_up = model.upsample.forward

    def up_hook(m):
        mm, aa = orig_up(m)
        captured["mels"], captured["aux"] = mm.detach().clone(), aa.detach().clone()
        return mm, aa

    model.upsample.forward = up_hook
    t0 = time.time()
    with NoiseInjector(fv, d.mode, noise) as inj:
        out = model.generate(torch.from_numpy(mel)[None], "/dev/null", batched, target, overlap, mu_law)
    dt = time.time() - t0
    assert inj.t == Lf, (inj.t, Lf)
    up_m = captured["mels"][0].numpy()
    up_a = captured["aux"][0].numpy()
    assert up_m.shape == (L, d.feat_dims)
    rec = dict(kind="gen", mode=d.mode, T=T, batched=batched, target=target, overlap=overlap,
               mu_law=mu_law, B=B, Lf=Lf, wseed=wseed, mseed=mseed, nseed=nseed, prune=prune,
               dims=np.array(repr(d)), ref_seconds=dt, state_sha=syn.state_digest(state),
               mel_sha=syn.digest(mel), noise_sha=syn.digest(noise),
               out_len=np.int64(len(out)), out_stride=np.int64(out_stride),
               output=np.asarray(out, dtype=np.float64)[::out_stride].copy(),
               out_sum=np.float64(np.asarray(out, dtype=np.float64).sum()),
               up_stride=cond_stride,
               up_mels=up_m[::cond_stride].copy(), up_aux=up_a[::cond_stride].copy(),
               up_mels_sum=np.float64(up_m.astype(np.float64).sum()),
               up_aux_sum=np.float64(up_a.astype(np.float64).sum()))
    raw = np.stack(inj.samples).T  # [B][Lf]
    raw = raw.astype(np.int16) if d.mode == "RAW" else raw.astype(np.float32)
    if raw_rows is None:
        rec["raw"] = raw
    else:
        rec["raw_rows"] = np.asarray(raw_rows, dtype=np.int64)
        rec["raw"] = raw[list(raw_rows)].copy()
        if raw_stride:
            rec["raw_stride"] = np.int64(raw_stride)
            rec["raw_strided"] = raw[:, ::raw_stride].copy()
    return rec


def gen_many_case(fv, name, d: syn.FatchordDims, T: int, n_utt: int, mseed0: int, target=11000,
                  overlap=550, mu_law=True, wseed=0, nseed=3, prune=0.0, out_stride=1):
    """A list of utterances vocoded ONE BY ONE by the reference generate(), as gen_wavernn.py:11-35
    does (unbatched, the mode config 4 times).  Utterance i: mel seed mseed0 + i, draws
    noise[:, i] of one [Lf][n_utt][K] array — the row order of a generate_many() launch over the
    same list.  Stores every utterance's float64 output (strided) and per-step loop outputs."""
    state = syn.make_fatchord_state(d, wseed)
    if prune > 0:
        from wavernn_amd.pruning import prune_state
        state = prune_state(state, prune)
    mels = [syn.make_mel(d.feat_dims, T, mseed0 + i) for i in range(n_utt)]
    L = d.hop_length * T
    noise = syn.make_noise(d.mode, n_utt, L, d.n_classes, nseed)
    model = build_ref_model(fv, d, state)
    outs, raws, dt = [], [], 0.0
    for i, mel in enumerate(mels):
        t0 = time.time()
        with NoiseInjector(fv, d.mode, noise[:, i:i + 1].copy()) as inj:
            out = model.generate(torch.from_numpy(mel)[None], "/dev/null", False, target, overlap, mu_law)
        dt += time.time() - t0
        assert inj.t == L, (inj.t, L)
        outs.append(np.asarray(out, dtype=np.float64))
        raws.append(np.stack(inj.samples).reshape(L))
    out = np.stack(outs)
    raw = np.stack(raws)
    raw = raw.astype(np.int16) if d.mode == "RAW" else raw.astype(np.float32)
    return dict(kind="gen_many", mode=d.mode, T=T, n_utt=n_utt, mseed0=mseed0, target=target,
                overlap=overlap, mu_law=mu_law, Lf=L, wseed=wseed, nseed=nseed, prune=prune,
                dims=np.array(repr(d)), ref_seconds=dt, state_sha=syn.state_digest(state),
                mel_sha=syn.digest(*mels), noise_sha=syn.digest(noise),
                out_len=np.int64(out.shape[1]), out_stride=np.int64(out_stride),
                output=out[:, ::out_stride].copy(), out_sum=out.sum(1), raw=raw)


# ---------------------------------------------------------------------- training forward
def train_case(fv, name, d: syn.FatchordDims, B=2, T=4, wseed=5, xseed=3, out_stride=1, n_grad=256):
    """The reference's teacher-forced forward (fatchord_version.py:131-167) and the backward of
    mean(y²) (§8(f)4): eval-mode output (BatchNorm running statistics), train-mode output (batch
    statistics), and per parameter the L2 norm and the first n_grad values of its gradient."""
    state = syn.make_fatchord_state(d, wseed)
    g = np.random.default_rng(xseed)
    mel = g.uniform(0, 1, (B, d.feat_dims, T + 2 * d.pad)).astype(np.float32)
    x = g.uniform(-1, 1, (B, T * d.hop_length)).astype(np.float32)
    model = build_ref_model(fv, d, state)
    t0 = time.time()
    model.eval()
    with torch.no_grad():
        y_eval = model(torch.from_numpy(x), torch.from_numpy(mel)).numpy()
    model.train()
    y = model(torch.from_numpy(x), torch.from_numpy(mel))
    loss = y.square().mean()
    loss.backward()
    dt = time.time() - t0
    rec = dict(kind="train", mode=d.mode, B=B, T=T, wseed=wseed, xseed=xseed, dims=np.array(repr(d)),
               ref_seconds=dt, state_sha=syn.state_digest(state), x_sha=syn.digest(mel, x),
               out_stride=np.int64(out_stride), y_eval=y_eval[:, ::out_stride].copy(),
               y_train=y.detach().numpy()[:, ::out_stride].copy(), loss=np.float64(loss.item()))
    names, norms, heads = [], [], []
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        gr = p.grad.detach().numpy().astype(np.float64).ravel()
        names.append(n)
        norms.append(np.sqrt((gr * gr).sum()))
        heads.append(np.pad(gr[:n_grad], (0, max(0, n_grad - gr.size))))
    rec["grad_names"] = np.array(names)
    rec["grad_norms"] = np.array(norms)
    rec["grad_heads"] = np.stack(heads).astype(np.float32)
    return rec


def cases():
    M, R = syn.DEFAULT_MOL, syn.DEFAULT_RAW
    return {
        # loop-level (C-ABI boundary) fixtures
        "loop_raw_b1": ("loop", dict(d=R, B=1, L=4400)),
        "loop_mol_b1": ("loop", dict(d=M, B=1, L=4400)),
        "loop_raw_b3": ("loop", dict(d=R, B=3, L=1500)),
        "loop_mol_b4": ("loop", dict(d=M, B=4, L=1500)),
        "loop_raw_tiny_b2": ("loop", dict(d=syn.TINY_RAW, B=2, L=3000)),
        "loop_mol_tiny_b2": ("loop", dict(d=syn.TINY_MOL, B=2, L=3000)),
        # config 1 (RAW 9-bit, rnn 512, 1 s) and its MoL twin, full length
        "loop_raw_1s": ("loop", dict(d=R, B=1, L=22275)),
        "loop_mol_1s": ("loop", dict(d=M, B=1, L=22275)),
        # config 4: rnn 896 with 95 % 4x4 block-sparse GRU weights; and a RAW twin at rnn 512
        "loop_mol_sparse896_b2": ("loop", dict(d=syn.SPARSE896_MOL, B=2, L=1100, prune=0.95)),
        "loop_raw_sparse_b2": ("loop", dict(d=R, B=2, L=1500, prune=0.95)),
        # end-to-end generate() fixtures
        "gen_mol_unbatched": ("gen", dict(d=M, T=22, batched=False, target=11000, overlap=550, mu_law=True)),
        "gen_raw_batched_mulaw": ("gen", dict(d=R, T=30, batched=True, target=2000, overlap=200, mu_law=True)),
        "gen_mol_batched": ("gen", dict(d=M, T=30, batched=True, target=1500, overlap=300, mu_law=True)),
        "gen_raw_tiny_unbatched": ("gen", dict(d=syn.TINY_RAW, T=24, batched=False, target=1000, overlap=100, mu_law=False)),
        # BASELINE sizes through the whole generate() (VERDICT r04 "do this" 1): config 1
        # exactly (RAW 9-bit, 1 s, unbatched), config 2 unbatched (the headline) and in the
        # reference's default fold-batched mode (hparams.py:58-60), config 3 (60 s, 115 folds)
        "gen_raw_1s_unbatched": ("gen", dict(d=R, T=81, batched=False, target=11000, overlap=550, mu_law=True)),
        "gen_mol_5s_unbatched": ("gen", dict(d=M, T=401, batched=False, target=11000, overlap=550,
                                             mu_law=True, cond_stride=275, out_stride=4)),
        "gen_mol_5s_batched": ("gen", dict(d=M, T=401, batched=True, target=11000, overlap=550,
                                           mu_law=True, cond_stride=275, out_stride=4)),
        "gen_mol_60s_batched": ("gen", dict(d=M, T=4811, batched=True, target=11000, overlap=550,
                                            mu_law=True, cond_stride=2750, out_stride=32,
                                            raw_rows=(0, 57, 114), raw_stride=50)),
        # config 4's production route (VERDICT r05 "do this" 1): the 95 %-pruned rnn-896 model
        # through the whole generate() — one 5 s utterance, and 8 shorter ones one by one
        # (gen_wavernn.py:11-35) for the 8-row generate_many launch bench.py times
        "gen_sparse896_5s_unbatched": ("gen", dict(d=syn.SPARSE896_MOL, T=401, batched=False, target=11000,
                                                   overlap=550, mu_law=True, cond_stride=275, out_stride=4,
                                                   prune=0.95)),
        "gen_sparse896_8utt": ("gen_many", dict(d=syn.SPARSE896_MOL, T=41, n_utt=8, mseed0=60, prune=0.95,
                                                out_stride=2)),
        # the training-side teacher-forced forward + backward (§8(f)4)
        "train_mol": ("train", dict(d=M, out_stride=2)),
        "train_raw": ("train", dict(d=R, out_stride=16)),
        # deepmind_version dual softmax (config 5 model), batch 1 as the reference generates
        "dm_b1": ("dm", dict(d=syn.DEFAULT_DM, L=2000)),
        "dm_tiny_b1": ("dm", dict(d=syn.TINY_DM, L=3000)),
    }


def main(argv):
    torch.set_num_threads(8)
    fv = import_reference()
    check_categorical_equivalence()
    todo = cases()
    names = argv or list(todo)
    for name in names:
        kind, kw = todo[name]
        fn = {"loop": loop_case, "gen": gen_case, "gen_many": gen_many_case, "dm": dm_case,
              "train": train_case}[kind]
        rec = fn(fv, name, **kw)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **{k: np.asarray(v) for k, v in rec.items()})
        print(f"{name}: {os.path.getsize(path) / 1024:.0f} KiB, reference {rec['ref_seconds']:.1f} s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
