"""A/B of bitset kernel variants in ONE process (interleaved rounds) on the
C2 workload; checks every variant's counts are identical to v1's."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import synth
n = int(os.environ.get("AB_N", "1000")); L = int(os.environ.get("AB_LEN", "2000000"))
variants = os.environ.get("AB_VARIANTS", "1,2").split(",")
rounds = int(os.environ.get("AB_ROUNDS", "5"))
ctx = gdist.Context(0)
g = synth.genomes(n, L, 0.002, 2)
blob, off = synth.to_blob(g); del g
sets = gdist.KmerSets.from_sequences([blob[off[i]:off[i + 1]] for i in range(n)], 21, gdist.KmerType.DNA, 0, ctx)
del blob
d, W = sets.build_bitsets()
print(f"n={n} L={L} dict={d} W={W}", flush=True)
dI = ctx.alloc(n * n * 4); dD = ctx.alloc(n * n * 8)
ref = None
times = {v: [] for v in variants}
for rnd in range(rounds):
    for v in variants:
        ctx.set_option("bitset_kernel", int(v))
        sets.matrix_device(dI.ptr, dD.ptr, n, (0, n), (0, n), upper=True, method=gdist.METHOD_BITSET)
        k_ms, call_ms, _ = ctx.last_timing()
        times[v].append(k_ms)
        if rnd == 0:
            I = dI.to_host(np.int32).reshape(n, n)
            iu = np.triu_indices(n, 1)
            if ref is None:
                ref = I[iu].copy()
            print(f"variant {v}: identical to first = {np.array_equal(I[iu], ref)}", flush=True)
pairs = n * (n - 1) // 2
for v in variants:
    t = np.array(times[v][1:] if len(times[v]) > 1 else times[v])
    wp = pairs * W / (t.min() * 1e-3)
    print(f"variant {v}: kernel ms median {np.median(t):.3f} min {t.min():.3f}  -> {pairs / (np.median(t) * 1e-3) / 1e6:.1f} M pairs/s, "
          f"{wp / 1e12:.2f} T word-pairs/s", flush=True)
