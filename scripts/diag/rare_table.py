"""Fused step (rare pairs in the chunk reduce) vs the rare kernel vs the
oracle on a C2-shaped collection: which pairs differ, by how much."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "genome.distance_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import gdist  # noqa: E402
import oracle  # noqa: E402
from gdist import synth  # noqa: E402

n, L = int(sys.argv[1]) if len(sys.argv) > 1 else 300, int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
seqs = [bytes(r) for r in synth.genomes(n, L, 0.002, 2)]
ctx = gdist.Context(0, {"trace": 1})
sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
sets.build_bitsets()
print("rare", sets.rare_info(), "sparse", sets.sparse_info(), flush=True)
I0, _ = sets.matrix(upper=False, method=gdist.METHOD_BITSET)
ctx.set_option("sparse_rare", 0)
I1, _ = sets.matrix(upper=False, method=gdist.METHOD_BITSET)
ctx.set_option("sparse_rare", None)
I2, _ = sets.matrix(upper=True, method=gdist.METHOD_BITSET)
off, codes = oracle.pack(seqs, 21, 0, 0)
eI, _ = oracle.matrix(off, codes, 0, n, 0, n, nthreads=16)
iu = np.triu_indices(n, 1)
for name, I in (("fused", I0), ("rare_kernel", I1), ("fused_upper", I2)):
    d = (I.astype(np.int64) - eI)[iu]
    bad = np.flatnonzero(d)
    print(name, "bad pairs", len(bad), "of", len(d), "diffs", np.unique(d[bad])[:10] if len(bad) else "", flush=True)
