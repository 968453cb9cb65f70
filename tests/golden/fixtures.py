"""Load a golden fixture and regenerate its inputs (weights, conditioning, mel, noise)
from the seeds it records, checking the SHA-256 digests made at generation time."""
from __future__ import annotations

import ast
import os

import numpy as np

from wavernn_amd import synthetic as syn

HERE = os.path.dirname(os.path.abspath(__file__))
LOOP_CASES = ["loop_raw_tiny_b2", "loop_mol_tiny_b2", "loop_raw_b1", "loop_mol_b1",
              "loop_raw_b3", "loop_mol_b4"]
LONG_LOOP_CASES = ["loop_raw_1s", "loop_mol_1s"]
SPARSE_LOOP_CASES = ["loop_mol_sparse896_b2", "loop_raw_sparse_b2"]
DM_CASES = ["dm_b1", "dm_tiny_b1"]
GEN_CASES = ["gen_mol_unbatched", "gen_raw_batched_mulaw", "gen_mol_batched", "gen_raw_tiny_unbatched"]
# generate() at BASELINE sizes (configs 1, 2 unbatched and fold-batched, 3), written by the
# reference itself; outputs stored strided / by row (make_golden.gen_case)
GEN_BASELINE_CASES = ["gen_raw_1s_unbatched", "gen_mol_5s_unbatched", "gen_mol_5s_batched", "gen_mol_60s_batched"]
# config 4's production route (rnn 896, 95 % 4x4 block-sparse GRU): one 5 s utterance through
# generate(), and 8 utterances vocoded one by one (the 8-row generate_many launch)
GEN_SPARSE_CASES = ["gen_sparse896_5s_unbatched"]
GEN_MANY_CASES = ["gen_sparse896_8utt"]

# MoL parity tolerance per sample under noise injection: ~50-100x the
# 5e-8..1.8e-7 the C restatement shows against the reference.
MOL_TOL = 1e-5


def load(name: str) -> dict:
    z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def dims_of(fx: dict):
    """The dims record make_golden stored (the repr of a frozen dataclass), parsed — never
    evaluated: one call of FatchordDims / DeepmindDims whose keyword values are literals."""
    text = str(fx["dims"])
    tree = ast.parse(text, mode="eval").body
    if not (isinstance(tree, ast.Call) and isinstance(tree.func, ast.Name) and not tree.args
            and tree.func.id in ("FatchordDims", "DeepmindDims")):
        raise ValueError(f"unexpected dims record {text!r}")
    kwargs = {kw.arg: ast.literal_eval(kw.value) for kw in tree.keywords}
    return getattr(syn, tree.func.id)(**kwargs)


def loop_inputs(fx: dict):
    d = dims_of(fx)
    B, L = int(fx["B"]), int(fx["L"])
    state = syn.make_fatchord_state(d, int(fx["wseed"]))
    if float(fx.get("prune", 0.0)) > 0:
        from wavernn_amd.pruning import prune_state
        state = prune_state(state, float(fx["prune"]))
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, int(fx["cseed"]))
    noise = syn.make_noise(d.mode, B, L, d.n_classes, int(fx["nseed"]))
    assert syn.state_digest(state) == str(fx["state_sha"]), "synthetic weight generator drifted"
    assert syn.digest(mels, aux) == str(fx["cond_sha"]), "synthetic conditioning drifted"
    assert syn.digest(noise) == str(fx["noise_sha"]), "synthetic noise drifted"
    return d, state, mels, aux, noise


def _state_of(fx: dict, d):
    state = syn.make_fatchord_state(d, int(fx["wseed"]))
    if float(fx.get("prune", 0.0)) > 0:
        from wavernn_amd.pruning import prune_state
        state = prune_state(state, float(fx["prune"]))
    return state


def gen_inputs(fx: dict):
    d = dims_of(fx)
    state = _state_of(fx, d)
    mel = syn.make_mel(d.feat_dims, int(fx["T"]), int(fx["mseed"]))
    noise = syn.make_noise(d.mode, int(fx["B"]), int(fx["Lf"]), d.n_classes, int(fx["nseed"]))
    assert syn.state_digest(state) == str(fx["state_sha"])
    assert syn.digest(mel) == str(fx["mel_sha"])
    assert syn.digest(noise) == str(fx["noise_sha"])
    return d, state, mel, noise


def gen_many_inputs(fx: dict):
    """(dims, state, mels [n_utt] of (feat, T), noise [Lf][n_utt][K]) of a `gen_many` fixture:
    utterance i was vocoded alone by the reference with draws noise[:, i]."""
    d = dims_of(fx)
    state = _state_of(fx, d)
    n, T = int(fx["n_utt"]), int(fx["T"])
    mels = [syn.make_mel(d.feat_dims, T, int(fx["mseed0"]) + i) for i in range(n)]
    noise = syn.make_noise(d.mode, n, int(fx["Lf"]), d.n_classes, int(fx["nseed"]))
    assert syn.state_digest(state) == str(fx["state_sha"])
    assert syn.digest(*mels) == str(fx["mel_sha"])
    assert syn.digest(noise) == str(fx["noise_sha"])
    return d, state, mels, noise


def dm_inputs(fx: dict):
    """(dims, state, noise [L][1][2Q]) of a deepmind fixture, regenerated and checked."""
    d = dims_of(fx)
    L = int(fx["L"])
    state = syn.make_deepmind_state(d, int(fx["wseed"]))
    noise = syn.make_dm_noise(1, L, d.quantisation, int(fx["nseed"]))
    assert syn.state_digest(state) == str(fx["state_sha"]), "synthetic weight generator drifted"
    assert syn.digest(noise) == str(fx["noise_sha"]), "synthetic noise drifted"
    return d, state, noise

TRAIN_CASES = ["train_mol", "train_raw"]


def train_inputs(fx: dict):
    """(dims, state, mel [B][feat][T + 2·pad], x [B][T·hop]) of a training-forward fixture."""
    d = dims_of(fx)
    state = syn.make_fatchord_state(d, int(fx["wseed"]))
    g = np.random.default_rng(int(fx["xseed"]))
    B, T = int(fx["B"]), int(fx["T"])
    mel = g.uniform(0, 1, (B, d.feat_dims, T + 2 * d.pad)).astype(np.float32)
    x = g.uniform(-1, 1, (B, T * d.hop_length)).astype(np.float32)
    assert syn.state_digest(state) == str(fx["state_sha"]), "synthetic weight generator drifted"
    assert syn.digest(mel, x) == str(fx["x_sha"]), "synthetic training inputs drifted"
    return d, state, mel, x
