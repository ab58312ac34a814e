"""Time hipMalloc / first touch / hipFree of large buffers (setup-path allocation churn)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
ctx = gdist.Context(0)
for gb in (1, 8, 16):
    for rep in range(3):
        t = time.perf_counter(); b = ctx.alloc(int(gb * 2**30)); ta = time.perf_counter() - t
        t = time.perf_counter(); b.from_host(np.zeros(1, np.uint8)); ctx.synchronize(); tt = time.perf_counter() - t
        t = time.perf_counter(); b.free(); tf = time.perf_counter() - t
        print(f"{gb:3d} GiB rep {rep}: alloc {ta*1e3:8.1f} ms  touch {tt*1e3:7.1f} ms  free {tf*1e3:8.1f} ms", flush=True)
# many live buffers then free all, then allocate again
bufs = [ctx.alloc(8 << 30) for _ in range(6)]
t = time.perf_counter()
for b in bufs: b.free()
print(f"free 6 x 8 GiB: {(time.perf_counter()-t)*1e3:.1f} ms")
t = time.perf_counter(); b = ctx.alloc(16 << 30); print(f"alloc 16 GiB after: {(time.perf_counter()-t)*1e3:.1f} ms"); b.free()
