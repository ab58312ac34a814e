"""Diagnostic (not collected by pytest): stage-by-stage check of the bitset path."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "genome.distance_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import gdist, oracle
from gdist import synth

def expected_bits(off, codes, keep):
    u, c = np.unique(codes, return_counts=True)
    d = u if keep else u[c >= 2]
    W = max(16, -(-(-(-len(d) // 64)) // 16) * 16)
    B = np.zeros((len(off) - 1, W), np.uint64)
    for s in range(len(off) - 1):
        cs = codes[off[s]:off[s + 1]]
        r = np.searchsorted(d, cs)
        ok = (r < len(d)) & (d[np.minimum(r, len(d) - 1)] == cs)
        r = r[ok]
        np.bitwise_or.at(B[s], r >> 6, np.left_shift(np.uint64(1), (r & 63).astype(np.uint64)))
    return d, B

ctx = gdist.Context(0)
for (n, L, p, k, cfg) in [(150, 5000, 0.01, 21, 92), (300, 3000, 0.05, 15, 91), (40, 2000, 0.05, 21, 5)]:
    seqs = [bytes(r) for r in synth.genomes(n, L, p, cfg)]
    off, codes = oracle.pack(seqs, k)
    eI, _ = oracle.matrix(off, codes, 0, n, 0, n)
    for keep in (False, True):
        sets = gdist.KmerSets.from_sequences(seqs, k, gdist.KmerType.DNA, 0, ctx)
        dsz, W = sets.build_bitsets(keep_singletons=keep)
        d, B = expected_bits(off, codes, keep)
        got = sets.bitsets()
        bad_rows = np.nonzero((got != B[:, :W]).any(axis=1))[0] if got.shape == B[:, :W].shape else "shape"
        print(f"n={n} k={k} keep={keep}: dict {dsz} vs {len(d)}, W {W} vs {B.shape[1]}, bad bit rows: "
              f"{bad_rows if isinstance(bad_rows, str) else (len(bad_rows), bad_rows[:10])}", flush=True)
        hostI = np.array([[int(np.bitwise_count(got[i] & got[j]).sum()) for j in range(n)] for i in range(n)])
        I, _ = sets.matrix(method=gdist.METHOD_BITSET)
        np.fill_diagonal(hostI, np.diag(eI))
        print(f"   tile kernel vs host popcount of device bits: mismatches {(I != hostI).sum()}; "
              f"vs oracle: {(I != eI).sum()}", flush=True)
        rows = np.nonzero((I != hostI).any(axis=1))[0]
        cols = np.nonzero((I != hostI).any(axis=0))[0]
        if len(rows):
            print("   bad rows", rows[:10], "...", rows[-5:], "bad cols", cols[:10], "...", cols[-5:], flush=True)
