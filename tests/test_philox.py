"""The numpy restatement of the in-kernel sampler draws (oracle/philox.py), on the CPU.

* Pinned to the published Philox-4x32-10 known-answer vectors (Salmon et al., SC'11; the same
  three vectors the Random123 distribution's kat_vectors file lists for philox4x32_10).
* The keying and word selection the kernels use (wrnn_device.h philox_word: counter
  (k >> 2, step, row lo, row hi), key (seed lo, seed hi), word k & 3), element by element.
* The maps: U(1e-5, 1 - 1e-5) for MoL (utils/distribution.py:106,118) and Exp(1) for RAW /
  deepmind (Categorical.sample ≡ argmax(probs / q)): Kolmogorov-Smirnov and moment checks on
  a few hundred thousand draws, bounds, and no correlation across k, rows or steps.
The device side of the same contract is tests/test_gpu_philox.py."""
import numpy as np
import pytest
from scipy import stats

from oracle import philox as ph

# (counter c0..c3, key k0 k1) -> output, Philox-4x32-10
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF),
     (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_known_answer_vectors(ctr, key, want):
    got = ph.philox4x32(np.array(ctr, dtype=np.uint32), np.array(key, dtype=np.uint32))
    assert [int(v) for v in got] == list(want)


def test_words_keying_element_by_element():
    seed, row0 = (7 << 32) | 0x1234, (3 << 32) - 2          # rows straddle 2^32: both halves used
    w = ph.philox_words(seed, row0, rows=4, step0=(1 << 32) - 3, steps=3, K=11)
    assert w.shape == (3, 4, 11) and w.dtype == np.uint32
    for s in range(3):
        for j in range(4):
            row, step = row0 + j, ((1 << 32) - 3 + s) & 0xFFFFFFFF
            for k in range(11):
                ctr = np.array([k >> 2, step, row & 0xFFFFFFFF, row >> 32], dtype=np.uint32)
                key = np.array([seed & 0xFFFFFFFF, seed >> 32], dtype=np.uint32)
                assert w[s, j, k] == ph.philox4x32(ctr, key)[k & 3], (s, j, k)


def test_mol_map_constants_and_fma():
    # the fp32 constant the device folds (v_fmac with 0x3f7ffeb0, tools/isa.sh fatchord_xcdm.hip)
    a = np.float32(1.0) - np.float32(2e-5)
    assert a.view(np.uint32) == 0x3F7FFEB0
    w = np.array([0, 0xFF, 0x100, 0x7FFFFFFF, 0xFFFFFF00, 0xFFFFFFFF], dtype=np.uint32)
    u = ph.draws_from_words(w, mol=True)
    assert u[0] == np.float32(1e-5) and u[1] == u[0]        # low 8 bits unused
    # exact FMA, checked with integer arithmetic: a·m·2^-24 + c, one rounding to fp32
    from fractions import Fraction
    for wi, ui in zip(w, u):
        m = int(wi) >> 8
        exact = Fraction(float(a)) * m / 2 ** 24 + Fraction(float(np.float32(1e-5)))
        lo = np.nextafter(ui, np.float32(-1))
        hi = np.nextafter(ui, np.float32(2))
        assert abs(Fraction(float(ui)) - exact) <= abs(Fraction(float(lo)) - exact)
        assert abs(Fraction(float(ui)) - exact) <= abs(Fraction(float(hi)) - exact)
    assert float(u.max()) <= 1 - 1e-5 + 1e-7


def test_uniform_draws_distribution():
    u = ph.philox_draws(1234, 0, rows=64, step0=0, steps=400, K=11, mol=True).astype(np.float64)
    assert u.min() >= np.float32(1e-5) and u.max() <= 1 - 1e-5
    x = u.ravel()                                            # 281 600 draws
    lo, span = 1e-5, 1 - 2e-5
    ks = stats.kstest(x, "uniform", args=(lo, span))
    assert ks.pvalue > 1e-4, ks
    assert abs(x.mean() - 0.5) < 4 * np.sqrt(1 / 12 / x.size)
    assert abs(x.var() - span ** 2 / 12) < 2e-3
    # no structure across k, rows or steps
    for axis in (0, 1, 2):
        a = np.moveaxis(u, axis, 0)
        r = np.corrcoef(a[:-1].ravel(), a[1:].ravel())[0, 1]
        assert abs(r) < 0.01, (axis, r)


def test_exponential_draws_distribution():
    q = ph.philox_draws(99, 5, rows=8, step0=17, steps=64, K=512, mol=False).astype(np.float64)
    x = q.ravel()                                            # 262 144 draws
    assert np.isfinite(x).all() and x.min() > 0 and x.max() <= 24 * np.log(2) + 1e-6
    ks = stats.kstest(x, "expon")
    assert ks.pvalue > 1e-4, ks
    assert abs(x.mean() - 1) < 4 / np.sqrt(x.size)
    assert abs(x.var() - 1) < 0.02
    for axis in (0, 1, 2):
        a = np.moveaxis(q, axis, 0)
        r = np.corrcoef(a[:-1].ravel(), a[1:].ravel())[0, 1]
        assert abs(r) < 0.01, (axis, r)


def test_categorical_via_exponential_is_unbiased():
    """argmax(p / q) with these Exp(1) draws samples Categorical(p) (the reference sampler,
    fatchord_version.py:232-235): chi-square over 6 classes and 20 000 draws."""
    p = np.array([0.05, 0.1, 0.15, 0.2, 0.2, 0.3])
    q = ph.philox_draws(2024, 0, rows=1, step0=0, steps=20000, K=6, mol=False)[:, 0].astype(np.float64)
    lab = np.argmax(p[None] / q, axis=1)
    cnt = np.bincount(lab, minlength=6)
    chi = stats.chisquare(cnt, p * lab.size)
    assert chi.pvalue > 1e-4, (cnt, chi)


def test_seed_and_row_change_the_stream():
    a = ph.philox_words(1, 0, 2, 0, 4, 8)
    assert not np.array_equal(a, ph.philox_words(2, 0, 2, 0, 4, 8))
    assert not np.array_equal(a[:, 1], a[:, 0])
    assert np.array_equal(a[:, 1:], ph.philox_words(1, 1, 1, 0, 4, 8))   # row keyed globally
    assert np.array_equal(a[2:], ph.philox_words(1, 0, 2, 2, 2, 8))      # step keyed globally
