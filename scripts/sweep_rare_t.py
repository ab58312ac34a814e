"""Sweep the rare-tier threshold T on the C2 workload (one process): build
the tiers for each T, time the N×N step, check every T gives identical counts."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import synth
n = int(os.environ.get("SW_N", "1000")); L = int(os.environ.get("SW_LEN", "2000000"))
Ts = [int(x) for x in os.environ.get("SW_T", "0,3,6,12,25,50,100,250").split(",")]
ctx = gdist.Context(0)
ctx.set_option("step_timing", 1)     # graph-replayed steps record their kernel times too
g = synth.genomes(n, L, 0.002, 2)
blob, off = synth.to_blob(g); del g
seqs = [blob[off[i]:off[i + 1]] for i in range(n)]
dI = ctx.alloc(n * n * 4); dD = ctx.alloc(n * n * 8)
ref = None
iu = np.triu_indices(n, 1)
for T in Ts:
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    d, W = sets.build_bitsets(rare_threshold=T)
    thr, lists, recs = sets.rare_info()
    ts = []
    for r in range(4):
        sets.matrix_device(dI.ptr, dD.ptr, n, (0, n), (0, n), upper=True, method=gdist.METHOD_BITSET)
        ts.append(ctx.last_timing()[0])
    I = dI.to_host(np.int32).reshape(n, n)[iu]
    if ref is None: ref = I.copy()
    print(f"T={T:4d} dense={d:9d} W={W:7d} rare_lists={lists:9d} records={recs:10d} step_ms={min(ts[1:]):8.3f} "
          f"identical={np.array_equal(I, ref)}", flush=True)
    del sets
