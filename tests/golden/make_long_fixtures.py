"""Full-length fixtures for the two BASELINE configs that are checked only in part elsewhere
(VERDICT r03, weak 1): produced by the C ORACLE (oracle/wavernn_oracle.c), which is itself pinned
bit-exact / within 6.4e-8 to the reference's own generate() by the 16 reference fixtures
(make_golden.py, tests/test_oracle_golden.py).  Running the Python reference for 1.4 M row-steps
(config 3) or 110 k rnn-896 steps (config 4) would take hours; the oracle restates the same loop
(fatchord_version.py:201-229) in C.

    python tests/golden/make_long_fixtures.py [long_mol_fold115] [long_sparse896_5s]

* long_mol_fold115 — config 3's loop shape: 115 rows × 12 100 steps (a 60 s utterance's folds),
  MoL rnn 512, injected noise.  Stores rows 0, 7, 64, 114 at full length and EVERY row at every
  50th step (a row-wise sample of the whole launch).
* long_sparse896_5s — config 4's: one 5 s row (110 275 steps) of the rnn-896 model with its GRU
  matrices pruned to 95 % in 4×4 blocks (pruning.prune_state), full length.
Inputs are regenerated from seeds (wavernn_amd.synthetic), SHA-256s stored as in make_golden.py.
The rows are independent, so the oracle runs over row chunks in parallel processes."""
from __future__ import annotations

import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402
from wavernn_amd import synthetic as syn  # noqa: E402
from wavernn_amd.pruning import prune_state  # noqa: E402

CASES = {
    "long_mol_fold115": dict(dims=syn.DEFAULT_MOL, B=115, L=12100, wseed=0, cseed=31, nseed=32, prune=0.0,
                             full_rows=(0, 7, 64, 114), sub=50),
    "long_sparse896_5s": dict(dims=syn.SPARSE896_MOL, B=1, L=110275, wseed=0, cseed=41, nseed=42, prune=0.95,
                              full_rows=(0,), sub=50),
}


def _state(c):
    st = syn.make_fatchord_state(c["dims"], c["wseed"])
    return prune_state(st, c["prune"]) if c["prune"] else st


def _chunk(args):
    name, b0, b1 = args
    c = CASES[name]
    d = c["dims"]
    mels, aux = syn.make_conditioning(c["B"], c["L"], d.feat_dims, d.res_out_dims, c["cseed"])
    noise = syn.make_noise(d.mode, c["B"], c["L"], d.n_classes, c["nseed"])
    out, _ = oracle.fatchord_loop(_state(c), d.mode, mels[b0:b1], aux[b0:b1], noise[:, b0:b1])
    return b0, out


def make(name: str, workers: int = 6) -> None:
    c = CASES[name]
    d = c["dims"]
    oracle.build()
    t = time.time()
    step = max(1, -(-c["B"] // workers))
    jobs = [(name, b0, min(c["B"], b0 + step)) for b0 in range(0, c["B"], step)]
    out = np.zeros((c["B"], c["L"]), np.float32)
    with ProcessPoolExecutor(max_workers=min(workers, len(jobs))) as ex:
        for b0, o in ex.map(_chunk, jobs):
            out[b0:b0 + o.shape[0]] = o
    mels, aux = syn.make_conditioning(c["B"], c["L"], d.feat_dims, d.res_out_dims, c["cseed"])
    noise = syn.make_noise(d.mode, c["B"], c["L"], d.n_classes, c["nseed"])
    st = _state(c)
    rows = np.array(c["full_rows"], np.int32)
    np.savez(os.path.join(HERE, name + ".npz"), dims=np.array(repr(d)), B=c["B"], L=c["L"], wseed=c["wseed"],
             cseed=c["cseed"], nseed=c["nseed"], prune=c["prune"], sub=c["sub"], full_rows=rows,
             out_full=out[rows], out_sub=out[:, ::c["sub"]], state_sha=syn.state_digest(st),
             cond_sha=syn.digest(mels, aux), noise_sha=syn.digest(noise), source=np.array("C oracle"))
    print(f"{name}: {c['B']} x {c['L']} in {time.time() - t:.0f} s")


if __name__ == "__main__":
    for n in (sys.argv[1:] or list(CASES)):
        make(n)
