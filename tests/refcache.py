"""The oracle's whole N x N matrix of a test collection, computed once and
sliced (test infrastructure: the checker). Parametrized tests that walk one
module-scoped collection through many options each used to recompute the
oracle over their regions — most of their time; the upper triangle is
computed once here (threaded C, oracle.matrix), mirrored (I and the
distance expression are symmetric in the two sets) and the diagonal filled
with |A| and the Java expression for (A, A)."""
import numpy as np

import oracle

_CACHE = {}


def full(off, codes):
    key = id(codes)
    hit = _CACHE.get(key)
    if hit is not None and hit[0] is codes:
        return hit[1], hit[2]
    n = len(off) - 1
    I, D = oracle.matrix(off, codes, 0, n, 0, n, flags=0x100, nthreads=8)
    I = I + I.T
    D = D + D.T
    sizes = np.diff(np.asarray(off, np.int64))
    idx = np.arange(n)
    I[idx, idx] = sizes
    D[idx, idx] = [oracle.distance(int(s), int(s), int(s)) for s in sizes]
    _CACHE[key] = (codes, I, D)
    return I, D


def matrix(off, codes, r0, r1, c0, c1, flags=0, nthreads=0):
    """oracle.matrix's result for the region (flags 0 or GDIST_UPPER_TRIANGLE:
    the pairs j <= i then hold 0, as the oracle leaves them)."""
    assert flags in (0, 0x100), flags
    fI, fD = full(off, codes)
    I = fI[r0:r1, c0:c1].copy()
    D = fD[r0:r1, c0:c1].copy()
    if flags & 0x100:
        low = np.fromfunction(lambda a, b: (c0 + b) <= (r0 + a), (r1 - r0, c1 - c0))
        I[low] = 0
        D[low] = 0.0
    return I, D
