import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "genome.distance_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import gdist, oracle
from gdist import synth
ctx = gdist.Context.default(0)
seqs = [bytes(r) for r in synth.genomes(300, 3000, 0.05, 91)]
def work(tag):
    for method in ["sorted", "bitset"]:
        sets = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
        if method != "sorted": sets.build_bitsets()
        sets.matrix(method=gdist.METHOD_SORTED if method == "sorted" else gdist.METHOD_BITSET)
        del sets
s2 = [bytes(r) for r in synth.genomes(150, 5000, 0.01, 92)]
off, codes = oracle.pack(s2, 21)
for trial in range(4):
    work(trial)
    a = gdist.KmerSets.from_sequences(s2, 21, gdist.KmerType.DNA, 0, ctx)
    oa, ca = a.download()
    ok = np.array_equal(oa, off) and np.array_equal(ca, codes)
    if not ok:
        sz = np.diff(oa); esz = np.diff(off)
        bad = np.nonzero(sz != esz)[0]
        print(f"trial {trial}: BAD total {len(ca)} vs {len(codes)}; sets with wrong size {len(bad)} first {bad[:8]} "
              f"sizes {sz[bad[:4]]} vs {esz[bad[:4]]}", flush=True)
        if len(bad) == 0:
            d = np.nonzero(ca != codes)[0]
            print("   same sizes, differing codes at", d[:10], len(d), flush=True)
    else:
        print(f"trial {trial}: ok", flush=True)
    b = gdist.KmerSets.from_sequences(s2, 21, gdist.KmerType.DNA, 0, ctx)
    ob, cb = b.download()
    print(f"   second pack ok: {np.array_equal(ob, off) and np.array_equal(cb, codes)}", flush=True)
    del a, b
