"""wrnn_device.h:label_x — c / 127.5 − 1 for the deepmind labels c ∈ {0..255} as c·r corrected by one
FMA (r = fl(1/127.5)) — equals the IEEE float32 quotient minus one for every label.  Exact
arithmetic (fractions) with float32 round-to-nearest-even after each operation."""
from fractions import Fraction

import numpy as np


def _rne32(fr: Fraction) -> Fraction:
    f = np.float32(float(fr))
    cands = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]
    best = min(cands, key=lambda c: (abs(Fraction(float(c)) - fr),
                                     int(np.frombuffer(np.float32(c).tobytes(), np.uint32)[0]) & 1))
    return Fraction(float(best))


def test_label_x_equals_ieee_division():
    r = _rne32(Fraction(1) / Fraction(255, 2))
    assert float(r) == float(np.float32(1.0) / np.float32(127.5))
    for c in range(256):
        want = _rne32(_rne32(Fraction(c) / Fraction(255, 2)) - 1)
        q0 = _rne32(Fraction(c) * r)
        e = _rne32(Fraction(c) - q0 * Fraction(255, 2))        # fma(-q0, 127.5, c)
        got = _rne32(_rne32(e * r + q0) - 1)                      # fma(e, r, q0) − 1
        assert got == want, c
        assert float(want) == float(np.float32(c) / np.float32(127.5) - np.float32(1.0))
