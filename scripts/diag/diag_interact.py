"""Diagnostic: reproduce rectangles -> prune interaction with state checks."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "genome.distance_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts", "diag")]
import numpy as np
import gdist, oracle
from gdist import synth
from diag_bitset import expected_bits  # noqa

ctx = gdist.Context.default(0)
seqs = [bytes(r) for r in synth.genomes(300, 3000, 0.05, 91)]
for method in ["sorted", "bitset", "bitset_keep"]:
    sets = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
    m = gdist.METHOD_SORTED
    if method != "sorted":
        sets.build_bitsets(keep_singletons=(method == "bitset_keep")); m = gdist.METHOD_BITSET
    for reg in [(0, 300, 0, 300, True), (0, 300, 0, 300, False), (37, 201, 5, 290, False), (100, 101, 0, 300, False),
                (129, 260, 0, 300, True), (0, 1, 0, 1, False)]:
        r0, r1, c0, c1, up = reg
        sets.matrix((r0, r1), (c0, c1), upper=up, method=m)
    print("rect", method, "done", flush=True)
    del sets

s2 = [bytes(r) for r in synth.genomes(150, 5000, 0.01, 92)]
off, codes = oracle.pack(s2, 21)
eI, _ = oracle.matrix(off, codes, 0, 150, 0, 150)
a = gdist.KmerSets.from_sequences(s2, 21, gdist.KmerType.DNA, 0, ctx)
b = gdist.KmerSets.from_sequences(s2, 21, gdist.KmerType.DNA, 0, ctx)
oa, ca = a.download(); ob, cb = b.download()
print("packed ok:", np.array_equal(oa, off) and np.array_equal(ca, codes), np.array_equal(cb, codes), flush=True)
a.build_bitsets(False)
_, Ba = expected_bits(off, codes, False)
print("a bits ok after build:", np.array_equal(a.bitsets(), Ba[:, :a.bitset_info()[1]]), flush=True)
b.build_bitsets(True)
_, Bb = expected_bits(off, codes, True)
print("b bits ok after build:", np.array_equal(b.bitsets(), Bb[:, :b.bitset_info()[1]]),
      "a bits still ok:", np.array_equal(a.bitsets(), Ba[:, :a.bitset_info()[1]]), flush=True)
Ia, _ = a.matrix(method=gdist.METHOD_BITSET)
print("Ia ok", np.array_equal(Ia, eI), "mismatch", (Ia != eI).sum(), flush=True)
Ib, _ = b.matrix(method=gdist.METHOD_BITSET)
print("Ib ok", np.array_equal(Ib, eI), "mismatch", (Ib != eI).sum(), flush=True)
print("after: a bits ok", np.array_equal(a.bitsets(), Ba[:, :a.bitset_info()[1]]),
      "b bits ok", np.array_equal(b.bitsets(), Bb[:, :b.bitset_info()[1]]), flush=True)
