"""Times the C2 sparse tile kernel (HIP events, option time_kernels) in the
product build ("base") or a diagnostic build of scripts/r05/diag_build.py
(its package copy first on sys.path). Diagnostic counts are wrong by design;
the base build's are checked against themselves only. Usage:
  python scripts/r05/diag_run.py base|d1|d2|... [reps]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
v = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
if v == "base":
    sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
else:
    sys.path.insert(0, os.path.join(ROOT, "scripts", "r05", "build", f"diag_{v}"))
    sys.path.append(os.path.join(ROOT, "genome.distance_amd"))      # synth
import numpy as np
import gdist
from gdist import synth
assert v == "base" or "diag_" in gdist.__file__, gdist.__file__
n = int(os.environ.get("DIAG_N", "1000"))
ctx = gdist.Context(0)
g = synth.genomes(n, 2_000_000, 0.002, 2)
blob, off = synth.to_blob(g); del g
sets = gdist.KmerSets.from_sequences([blob[off[i]:off[i + 1]] for i in range(n)], 21, gdist.KmerType.DNA, 0, ctx)
del blob
sets.build_bitsets()
for kv in os.environ.get("DIAG_OPTS", "").split(","):
    if kv:
        k, x = kv.split("=")
        ctx.set_option(k, int(x))
dI, dD = ctx.alloc(n * n * 4), ctx.alloc(n * n * 8)
ctx.set_option("time_kernels", 1)
ks = []
for r in range(reps):
    sets.matrix_device(dI.ptr, dD.ptr, n, (0, n), (0, n), upper=True, method=gdist.METHOD_BITSET)
    ctx.synchronize()
    ks.append(ctx.kernel_ms("sparse"))
ks = np.array(ks[2:])
print(f"{v} {os.environ.get('DIAG_OPTS', '')}: sparse kernel ms median {np.median(ks):.4f} min {ks.min():.4f} max {ks.max():.4f}",
      flush=True)
