import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "genome.distance_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import gdist, oracle
from gdist import synth
ctx = gdist.Context.default(0)
seqs = [bytes(r) for r in synth.genomes(300, 3000, 0.05, 91)]
s2 = [bytes(r) for r in synth.genomes(150, 5000, 0.01, 92)]
off, codes = oracle.pack(s2, 21)
for trial in range(8):
    for method in ["sorted", "bitset"]:
        sets = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
        if method != "sorted": sets.build_bitsets()
        sets.matrix(method=gdist.METHOD_SORTED if method == "sorted" else gdist.METHOD_BITSET)
        del sets
    a = gdist.KmerSets.from_sequences(s2, 21, gdist.KmerType.DNA, 0, ctx)
    o1, c1 = a.download()
    time.sleep(0.5)
    ctx.synchronize()
    o2, c2 = a.download()
    ok1 = np.array_equal(c1, codes); ok2 = np.array_equal(c2, codes)
    msg = f"trial {trial}: first download ok={ok1} second download ok={ok2}"
    if not ok1:
        d = np.nonzero(c1 != codes)[0]
        msg += f" | bad from {d[0]} n={len(d)} zeros_in_bad={int((c1[d] == 0).sum())} c1==c2:{np.array_equal(c1, c2)}"
        # are bad values codes from elsewhere in the expected array?
        msg += f" bad_vals_in_expected={np.isin(c1[d[:1000]], codes).mean():.2f}"
    print(msg, flush=True)
    del a
