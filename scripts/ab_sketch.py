"""A/B of sketch kernels in ONE process: variants are '+'-joined parts, kN
(option sketch_k), tN (sketch_tile) or name=value (any option, e.g.
sketch_phase=0, sketch_cap=200; "default" = no options), on the C5 workload: every variant's common
counts on a row block are checked identical to the first variant's, then the
full upper triangle is timed in interleaved rounds."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import synth

n = int(os.environ.get("AB_N", "50000")); L = int(os.environ.get("AB_LEN", "100000"))
width = int(os.environ.get("AB_WIDTH", "1000"))
variants = os.environ.get("AB_VARIANTS", "default,sketch_phase=0").split(",")
rounds = int(os.environ.get("AB_ROUNDS", "3"))
check_rows = min(n, 2048)


KNOBS = ("sketch_tile", "sketch_k", "sketch_phase", "sketch_cap", "sketch_v2", "sketch_ring", "sketch_wait", "sketch_perm")


def apply(v):
    for k in KNOBS:
        ctx.set_option(k, None)
    for part in v.split("+"):
        if "=" in part:
            name, val = part.split("=")
            ctx.set_option(name, int(val))
        elif part == "default":
            pass
        elif part.startswith("k"):
            ctx.set_option("sketch_k", int(part[1:]))
        elif part.startswith("t"):
            ctx.set_option("sketch_tile", int(part[1:]))




ctx = gdist.Context(0)
t = time.time()
g = synth.genomes(n, L, 0.05, 5)
blob, off = synth.to_blob(g); del g
sets = gdist.KmerSets.from_sequences([blob[off[i]:off[i + 1]] for i in range(n)], 21, gdist.KmerType.DNA, 0, ctx)
del blob
sk = sets.sketches(width)
del sets
print(f"n={n} L={L} width={width} setup {time.time() - t:.1f}s", flush=True)
dC = ctx.alloc(n * n * 4)
ref = None
for v in variants:
    apply(v)
    for fl in (0, gdist.SKETCH_JACCARD):
        sk.matrix_device(dC.ptr, None, n, (0, check_rows), (0, n), upper=True, flags=fl)
        C = dC.to_host(np.int32, check_rows * n).reshape(check_rows, n)
        C = np.triu(C, 1)
        if ref is None:
            ref = {}
        if fl not in ref:
            ref[fl] = C.copy()
        print(f"{v} flags={fl:#x}: identical to {variants[0]} = {np.array_equal(C, ref[fl])}", flush=True)
times = {v: [] for v in variants}
for rnd in range(rounds):
    for v in variants:
        apply(v)
        sk.matrix_device(dC.ptr, None, n, (0, n), (0, n), upper=True)
        times[v].append(ctx.last_timing()[0])
pairs = n * (n - 1) // 2
for v in variants:
    tt = np.array(times[v])
    print(f"{v}: kernel ms median {np.median(tt):.1f} min {tt.min():.1f} -> "
          f"{pairs / (np.median(tt) * 1e-3) / 1e9:.3f} G pairs/s", flush=True)
