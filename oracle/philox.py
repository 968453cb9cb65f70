"""Oracle: numpy restatement of the in-kernel sampler draws (noise == NULL).

TEST INFRASTRUCTURE ONLY — imported by tests/ as the checker of the device's Philox stream
(`philox_word` / `philox_noise`, wavernn_amd/csrc/wrnn_device.h; materialised by the C-ABI entry
`wrnn_philox_draws`), never by the product package.

The generator is the published Philox-4x32-10 counter-based RNG (J. Salmon, M. Moraes, R. Dror,
D. Shaw, "Parallel Random Numbers: As Easy as 1, 2, 3", SC'11; the Random123 library's
philox4x32_R with R = 10), written here from the paper's round function:
    (hi0, lo0) = mulhilo(0xD2511F53, c0);  (hi1, lo1) = mulhilo(0xCD9E8D57, c2)
    c' = (hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0);  key += (0x9E3779B9, 0xBB67AE85)
pinned by the paper's known-answer vectors (tests/test_philox.py).

Keying (shard-invariant draws): draw k of global row `row` at loop step `step`
is word (k & 3) of Philox(counter = (k >> 2, step, row & 0xffffffff, row >> 32),
key = (seed & 0xffffffff, seed >> 32)).  Its top 24 bits m give
  * MoL  (utils/distribution.py:106,118, u ~ U(1e-5, 1 - 1e-5)): fma(1 - 2e-5, m·2^-24, 1e-5) in fp32;
    the product of two fp32 values is exact in float64 and the sum too (it spans < 53 bits:
    2^0 .. 2^-48), so one rounding to fp32 is the FMA exactly;
  * RAW / deepmind (q ~ Exp(1); Categorical.sample ≡ argmax(probs / q),
    fatchord_version.py:232-235, deepmind_version.py:130,150): -log((m + 1)·2^-24) in float64,
    rounded once to fp32, as the device computes it (two faithfully rounded float64 logs round
    to different fp32 values only across a rounding boundary, ~2^-29 per draw; the tests state
    the bound they check — observed bit-equal on every draw).
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)
_S32 = np.uint64(32)


def philox4x32(ctr, key, rounds: int = 10) -> np.ndarray:
    """Philox-4x32-R of counters `ctr` [..., 4] under keys `key` [..., 2] (uint32, broadcast)
    → [..., 4] uint32."""
    ctr = np.asarray(ctr, dtype=np.uint32)
    key = np.asarray(key, dtype=np.uint32)
    shape = np.broadcast_shapes(ctr.shape[:-1], key.shape[:-1])
    c = [np.broadcast_to(ctr[..., i], shape).astype(np.uint64) for i in range(4)]
    k0 = np.broadcast_to(key[..., 0], shape).astype(np.uint32)
    k1 = np.broadcast_to(key[..., 1], shape).astype(np.uint32)
    for _ in range(rounds):
        p0 = M0 * c[0]          # < 2^64: exact in uint64
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> _S32, p0 & _MASK
        hi1, lo1 = p1 >> _S32, p1 & _MASK
        c = [hi1 ^ c[1] ^ k0.astype(np.uint64), lo1, hi0 ^ c[3] ^ k1.astype(np.uint64), lo0]
        with np.errstate(over="ignore"):
            k0 = k0 + W0
            k1 = k1 + W1
    return np.stack([x.astype(np.uint32) for x in c], axis=-1)


def philox_words(seed: int, row0: int, rows: int, step0: int, steps: int, K: int) -> np.ndarray:
    """The 32-bit words behind draws [steps][rows][K] of rows row0.. at steps step0.."""
    seed &= (1 << 64) - 1
    t = (np.arange(steps, dtype=np.uint64) + np.uint64(step0)).astype(np.uint32)
    r = np.arange(rows, dtype=np.uint64) + np.uint64(row0 & ((1 << 64) - 1))
    k = np.arange(K, dtype=np.uint32)
    nq = (K + 3) // 4
    T, R, Q = np.meshgrid(t, r, np.arange(nq, dtype=np.uint32), indexing="ij")
    ctr = np.stack([Q, T, (R & _MASK).astype(np.uint32), (R >> _S32).astype(np.uint32)], axis=-1)
    key = np.array([seed & 0xFFFFFFFF, seed >> 32], dtype=np.uint32)
    out = philox4x32(ctr, key)                            # [steps][rows][nq][4]
    return np.ascontiguousarray(out.reshape(steps, rows, nq * 4)[:, :, k])


def draws_from_words(w: np.ndarray, mol: bool) -> np.ndarray:
    """The fp32 draws of words w (see the module docstring for the maps)."""
    m = (np.asarray(w, dtype=np.uint32) >> np.uint32(8)).astype(np.float64)
    if mol:
        a = float(np.float32(1.0) - np.float32(2e-5))       # fp32 constant, as the device folds it
        u = m * 2.0 ** -24                                  # exact: the device's (float)m · 2^-24
        return (a * u + float(np.float32(1e-5))).astype(np.float32)   # exact sum, one rounding
    return (-np.log((m + 1.0) * 2.0 ** -24)).astype(np.float32)


def philox_draws(seed: int, row0: int, rows: int, step0: int, steps: int, K: int, mol: bool) -> np.ndarray:
    """Draws [steps][rows][K] exactly as wrnn_philox_draws lays them out (the noise == NULL draws
    of every loop kernel; usable as injected `noise`)."""
    return np.ascontiguousarray(draws_from_words(philox_words(seed, row0, rows, step0, steps, K), mol))
