"""Device memory at each stage of the C5 setup (hipMemGetInfo via ctypes):
where the full-size C5 test ran out of memory."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "genome.distance_amd")]
import numpy as np  # noqa: E402

import gdist  # noqa: E402
from gdist import synth  # noqa: E402

hip = C.CDLL("libamdhip64.so")


def mem(tag):
    f, t = C.c_size_t(), C.c_size_t()
    hip.hipMemGetInfo(C.byref(f), C.byref(t))
    print(f"{tag:32s} free {f.value / 2**30:8.1f} GiB of {t.value / 2**30:.1f}", flush=True)


n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
ctx = gdist.Context(0, {"trace": 1})
mem("start")
t = time.time()
blob, off = synth.to_blob(synth.genomes(n, 100_000, 0.05, 5))
print(f"generate {time.time() - t:.1f} s", flush=True)
sets = gdist.KmerSets.from_blob(blob, off, 21, gdist.KmerType.DNA, 0, ctx)
mem("after pack")
sk = sets.sketches(1000)
mem("after sketches")
del sets
mem("after del sets")
dC = ctx.alloc(n * n * 4)
mem("after alloc C")
dD = ctx.alloc(n * n * 8)
mem("after alloc D")
