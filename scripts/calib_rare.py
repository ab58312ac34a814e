"""Rare-tier kernel calibration: one collection, one row block, both rare
kernels (list-major rare_pairs_kernel, row-major rare_rows_kernel) run in line
after the dense tile launches. Run under `rocprofv3 --kernel-trace --stats`;
the per-kernel averages of the stats file, with the tier statistics printed
here, fit the cost model in gdist_internal.hpp (scripts/calib_rare.sh).

  CAL_CASE  c2 | c3 | c4s (C4 slice, 10k genomes) | g8 (C2 weak scaling at 8 ranks, N=2828)
  CAL_T     forced rare threshold (-1: the cost model's)
  CAL_ROWS  "a:b" row block as fractions of N (default 0:1, the whole triangle)
"""
import json, math, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import gdist
from gdist import synth

CASES = {
    "c2": dict(n=1000, length=2_000_000, p_max=0.002, protein=False, k=21, cfg=2),
    "c3": dict(n=10000, length=33_333, p_max=0.10, protein=True, k=8, cfg=3),
    "c4s": dict(n=10000, length=100_000, p_max=0.05, protein=False, k=21, cfg=4),
    "g8": dict(n=int(round(1000 * math.sqrt(8))), length=2_000_000, p_max=0.002, protein=False, k=21, cfg=2),
}
case = os.environ.get("CAL_CASE", "c2")
c = CASES[case]
N = c["n"]
ctx = gdist.Context(0)
ctx.set_option("step_timing", 1)     # graph-replayed steps record their kernel times too
t = time.time()
g = synth.genomes(N, c["length"], c["p_max"], c["cfg"], protein=c["protein"])
blob, off = synth.to_blob(g); del g
kind = gdist.KmerType.PROT if c["protein"] else gdist.KmerType.DNA
sets = gdist.KmerSets.from_sequences([blob[off[i]:off[i + 1]] for i in range(N)], c["k"], kind, 0, ctx)
del blob
dsz, W = sets.build_bitsets(rare_threshold=int(os.environ.get("CAL_T", "-1")))
T, lists, recs = sets.rare_info()
incs, max_list = sets.rare_stats()
a, b = (float(x) for x in os.environ.get("CAL_ROWS", "0:1").split(":"))
r0, r1 = int(round(a * N)), int(round(b * N))
dI, dD = ctx.alloc((r1 - r0) * N * 4), ctx.alloc((r1 - r0) * N * 8)
ctx.set_option("rare_overlap", 0)
ms = {}
for kern in ("0", "1"):
    ctx.set_option("rare_kernel", int(kern))
    for _ in range(4):
        sets.matrix_device(dI.ptr, dD.ptr, N, (r0, r1), (0, N), upper=True, method=gdist.METHOD_BITSET)
    ctx.synchronize()
    ms[kern] = ctx.last_timing()[0]
print(json.dumps(dict(case=case, n=N, rows=[r0, r1], W=W, dict=dsz, T=T, lists=lists, records=recs, incs=incs,
                      max_list=max_list, setup_s=round(time.time() - t, 1),
                      kernel_ms_last={"list": ms["0"], "row": ms["1"]})), flush=True)
