"""Per-rank step time of the row-sharded C2 weak-scaling run, emulated on one
GPU: the G-rank collection (N = 1000 sqrt(G)) is built once and each rank's
triangle row block is timed alone (list-major vs row-major rare kernel)."""
import math, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import shard, synth

G = int(os.environ.get("EMU_G", "8"))
N = int(round(1000 * math.sqrt(G)))
ctx = gdist.Context(0, options=gdist.kmers.options_from_env())   # GDIST_<NAME> A/B switches
t = time.time()
g = synth.genomes(N, 2_000_000, 0.002, 2)
blob, off = synth.to_blob(g); del g
sets = gdist.KmerSets.from_sequences([blob[off[i]:off[i + 1]] for i in range(N)], 21, gdist.KmerType.DNA, 0, ctx)
del blob
T_force = int(os.environ.get("EMU_T", "-1"))
dsz, W = sets.build_bitsets(rare_threshold=T_force)
T, lists, recs = sets.rare_info()
print(f"G={G} N={N} setup {time.time() - t:.1f}s dict={dsz} W={W} rare T={T} lists={lists} records={recs}", flush=True)
bounds = shard.triangle_bounds(N, G, int(os.environ.get("EMU_ALIGN", "1")))
incs, max_list = sets.rare_stats()
print(f"rare incs {incs} longest list {max_list}", flush=True)
if os.environ.get("EMU_BALANCE", "1") == "1":
    bounds = shard.balanced_bounds(N, G, lambda a, b: sets.block_cost((a, b))[0])
model = [sets.block_cost((bounds[g], bounds[g + 1])) for g in range(G)]
print("modelled per-rank ms / rare kernel: " + str([(round(t * 1e3, 2), k) for t, k in model]), flush=True)
assert len(bounds) == G + 1 and bounds[0] == 0 and bounds[-1] == N and all(b <= c for b, c in zip(bounds, bounds[1:]))
max_rows = max(bounds[k + 1] - bounds[k] for k in range(G))      # the last rank has the most rows
dI, dD = ctx.alloc(max_rows * N * 4), ctx.alloc(max_rows * N * 8)
print(f"row blocks {bounds} (max {max_rows} rows; buffers {max_rows * N * 12 / 1e9:.2f} GB)", flush=True)
for kern in os.environ.get("EMU_KERNELS", ",0,1").split(","):   # "" = the model's per-block choice
    ctx.set_option("rare_kernel", int(kern) if kern else None)
    times = []
    for rk in range(G):
        r0, r1 = bounds[rk], bounds[rk + 1]
        assert (r1 - r0) * N * 4 <= dI.nbytes and (r1 - r0) * N * 8 <= dD.nbytes   # output fits (ld = N)
        for _ in range(3):   # plan build, graph capture (the process's first instantiation is slow), replay
            sets.matrix_device(dI.ptr, dD.ptr, N, (r0, r1), (0, N), upper=True, method=gdist.METHOD_BITSET)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            sets.matrix_device(dI.ptr, dD.ptr, N, (r0, r1), (0, N), upper=True, method=gdist.METHOD_BITSET)
        ctx.synchronize()
        times.append((time.perf_counter() - t0) / 20 * 1e3)
    pairs = N * (N - 1) // 2
    print(f"rare kernel {kern or 'auto'}: per-rank ms {[round(x, 2) for x in times]} -> max {max(times):.2f} ms, "
          f"emulated {pairs / (max(times) * 1e-3) / 1e6:.0f} M pairs/s on {G} GPUs "
          f"(balance {min(times) / max(times):.2f})", flush=True)
