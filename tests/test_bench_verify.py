"""bench.py's end-of-run verification: the independent numpy kmer recount
agrees with the oracle's packer, and verify_sample flags a wrong device
entry (CPU only: device buffers are faked)."""
import os
import sys

import numpy as np

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gdist import synth  # noqa: E402


def test_recount_matches_oracle_pack():
    for protein, k, kind in ((False, 21, 0), (True, 8, 1)):
        g = [bytes(r) for r in synth.genomes(4, 4000, 0.05, 7, protein=protein)]
        off, codes = oracle.pack(g, k, kind, 0)
        for i in range(len(g)):
            mine = bench._kmer_codes(g[i], k, protein)
            assert np.array_equal(mine, np.asarray(codes[off[i]:off[i + 1]], dtype=np.uint64))


class _FakeBuf:
    def __init__(self, arr):
        self.arr = arr

    def to_host(self, dtype, count=None, offset=0):
        return self.arr.view(dtype)[offset:offset + count].copy()

    def from_host(self, a, offset=0):
        self.arr[offset:offset + len(a)] = a


def test_verify_sample_detects_mismatch():
    cfg = dict(length=3000, p_max=0.01, cfg=2, k=21, protein=False)
    n = 6
    g = [bytes(r) for r in synth.genomes(n, cfg["length"], cfg["p_max"], cfg["cfg"])]
    off, codes = oracle.pack(g, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n)
    ident = lambda v: v   # noqa: E731  (single rank: max over ranks is the value)
    r0, r1 = 2, 5
    I = np.ascontiguousarray(eI[r0:r1].astype(np.int32)).ravel()
    D = np.ascontiguousarray(eD[r0:r1]).ravel()
    good = bench.verify_sample(cfg, "bitset", n, r0, r1, _FakeBuf(I), _FakeBuf(D), ident)
    assert good["ok"] and good["pairs_per_rank"] == 4
    bad_I = I.copy()
    bad_I[(2 - r0) * n + 3] += 1          # pair (2, 3) is the first one checked
    bad = bench.verify_sample(cfg, "bitset", n, r0, r1, _FakeBuf(bad_I), _FakeBuf(D), ident)
    assert not bad["ok"]
    assert bench.verify_sample(cfg, "sketch", n, r0, r1, None, None, ident) is None


def test_verify_sample_poisons_before_its_step():
    """The sampled pairs are poisoned before the verifying step: a step that
    rewrites them passes, one that skips them (a replay that dropped a
    kernel family) fails."""
    cfg = dict(length=3000, p_max=0.01, cfg=2, k=21, protein=False)
    n = 6
    g = [bytes(r) for r in synth.genomes(n, cfg["length"], cfg["p_max"], cfg["cfg"])]
    off, codes = oracle.pack(g, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n)
    ident = lambda v: v   # noqa: E731
    r0, r1 = 2, 5
    I = np.ascontiguousarray(eI[r0:r1].astype(np.int32)).ravel()
    D = np.ascontiguousarray(eD[r0:r1]).ravel()
    bI, bD = _FakeBuf(I.copy()), _FakeBuf(D.copy())

    def full_step():
        bI.arr[:] = I
        bD.arr[:] = D
    res = bench.verify_sample(cfg, "bitset", n, r0, r1, bI, bD, ident, step=full_step)
    assert res["ok"] and res["poisoned"]
    res = bench.verify_sample(cfg, "bitset", n, r0, r1, bI, bD, ident, step=lambda: None)
    assert not res["ok"]
