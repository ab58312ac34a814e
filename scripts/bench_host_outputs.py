"""PCIe-inclusive rate: the same all-pairs calls with host outputs (the
C-ABI copies I and D back), next to the device-resident timing."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import synth

ctx = gdist.Context(0)
for name, n, L, pmax, prot, k, sketch in [("c2", 1000, 2_000_000, 0.002, False, 21, 0), ("c3", 10000, 33_333, 0.10, True, 8, 0),
                                          ("c5 (n=20000)", 20000, 100_000, 0.05, False, 21, 1000)]:
    g = synth.genomes(n, L, pmax, 7, protein=prot)
    sets = gdist.KmerSets.from_sequences([bytes(r) for r in g], k, gdist.KmerType.PROT if prot else gdist.KmerType.DNA, 0, ctx)
    del g
    obj = sets.sketches(sketch) if sketch else sets
    if not sketch:
        sets.prepare()
    pairs = n * (n - 1) // 2
    dI, dD = ctx.alloc(n * n * 4), ctx.alloc(n * n * 8)
    obj.matrix_device(dI.ptr, dD.ptr, n, (0, n), (0, n), upper=True)
    ctx.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        obj.matrix_device(dI.ptr, dD.ptr, n, (0, n), (0, n), upper=True)
    ctx.synchronize()
    td = (time.perf_counter() - t) / 3
    obj.matrix(upper=True)
    t = time.perf_counter()
    obj.matrix(upper=True)
    th = time.perf_counter() - t
    print(f"{name}: device-resident {pairs / td / 1e6:.1f} M pairs/s ({td * 1e3:.1f} ms); host outputs I+D "
          f"({n * n * 12 / 1e9:.2f} GB) {pairs / th / 1e6:.1f} M pairs/s ({th * 1e3:.1f} ms)", flush=True)
    dI.free(); dD.free()
