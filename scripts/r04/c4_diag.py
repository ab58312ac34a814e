"""C4 on one GPU: pack, consuming code all-gather, then the bitset build
(METHOD_BITSET, option trace) with its stage timings on stderr; the error
if it fails. Then one 64-row slice through it."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import gdist  # noqa: E402
from gdist import synth  # noqa: E402

N = int(os.environ.get("C4_N", "100000"))
ctx = gdist.Context(0)
ctx.comm_init(gdist.Context.unique_id(), 1, 0)
g = synth.genomes(N, 100_000, 0.05, 4)
blob, off = synth.to_blob(g)
del g
local = gdist.KmerSets.from_blob(blob, off, 21, gdist.KmerType.DNA, 0, ctx)
del blob
gs = local.allgather(consume=True)
ctx.set_option("trace", 1)
for kv in os.environ.get("C4_OPTS", "").split(","):
    if kv:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
t = time.time()
try:
    m, cb, cs = gs.prepare(gdist.METHOD_BITSET)
    print(f"built in {time.time() - t:.1f} s: est bitset {cb:.4g} s sorted {cs:.4g} s; variant {gs.variant_info()}; "
          f"bitset {gs.bitset_info()}; rare {gs.rare_info()} {gs.rare_stats()}", flush=True)
except Exception as e:
    print(f"build failed after {time.time() - t:.1f} s: {e!r}", flush=True)
    sys.exit(1)
ctx.set_option("trace", 0)
for rows in ((0, 64), (64645, 64661)):
    t = time.time()
    gs.matrix(rows, (0, N), upper=True, method=gdist.METHOD_BITSET)
    print(f"rows {rows}: {time.time() - t:.3f} s, last timing {ctx.last_timing()}", flush=True)
ctx.comm_destroy()
