"""In-process A/B on the C4 slice (bench.py --config c4 --rows 0:1024
--force-exchange, built once): the code all-gather on a one-rank RCCL
communicator, METHOD_AUTO's three tiers, then per setting (AB_ENVS="k=v,k=v;..."
of context options, "" = defaults) interleaved rounds of the 1,024-row step:
the step's kernel span and, with serial_step = 1 and time_kernels = 1, each
kernel family alone (variant walk, MFMA tiles, rare walk). Every setting's
counts must equal the first one's."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import synth

N, L, P, CFG, K = 100_000, 100_000, 0.05, 4, 21
R0, R1 = 0, int(os.environ.get("AB_ROWS", "1024"))
settings = os.environ.get("AB_ENVS", "").split(";")
rounds = int(os.environ.get("AB_ROUNDS", "3"))
t0 = time.time()
ctx = gdist.Context(0)
ctx.comm_init(gdist.Context.unique_id(), 1, 0)
g = synth.genomes(N, L, P, CFG)
blob, off = synth.to_blob(g)
del g
local = gdist.KmerSets.from_blob(blob, off, K, gdist.KmerType.DNA, 0, ctx)
del blob
gs = local.allgather(consume=True)
chosen, _, _ = gs.prepare(gdist.METHOD_AUTO, pairs=float((R1 - R0) * N))
assert chosen == gdist.METHOD_BITSET
gs.release_codes()
print(f"built in {time.time() - t0:.1f} s; variant {gs.variant_info()}", flush=True)
rows = R1 - R0
dI, dD = ctx.alloc(rows * N * 4), ctx.alloc(rows * N * 8)
up = np.fromfunction(lambda i, j: j > i + R0, (rows, N))
ref = None
res = {s: {"span": [], "variant": [], "dense": [], "rare": []} for s in settings}
names = ["trace"] + sorted({kv.split("=")[0] for s in settings for kv in s.split(",") if kv})
base = {k: ctx.option(k) for k in names}
for rnd in range(rounds):
    for s in settings:
        for k, v in base.items():
            ctx.set_option(k, v)
        for kv in s.split(","):
            if kv:
                k, v = kv.split("=")
                ctx.set_option(k, int(v))
        ctx.set_option("step_timing", 1)
        for _ in range(2):
            gs.matrix_device(dI.ptr, dD.ptr, N, (R0, R1), (0, N), upper=True, method=gdist.METHOD_BITSET)
        ctx.synchronize()
        res[s]["span"].append(ctx.last_timing()[0])
        ctx.set_option("time_kernels", 1)
        ctx.set_option("serial_step", 1)
        gs.matrix_device(dI.ptr, dD.ptr, N, (R0, R1), (0, N), upper=True, method=gdist.METHOD_BITSET)
        ctx.synchronize()
        for f in ("variant", "dense", "rare"):
            res[s][f].append(ctx.kernel_ms(f))
        ctx.set_option("time_kernels", None)
        ctx.set_option("serial_step", None)
        if rnd == 0 and "=9" not in s:      # an option at 9: a timing-only experiment (counts differ)
            I = dI.to_host(np.int32, rows * N).reshape(rows, N)[up]
            if ref is None:
                ref = I.copy()
            else:
                assert np.array_equal(I, ref), f"setting {s!r}: counts differ"
for s in settings:
    r = res[s]
    print(f"[{s or 'default'}] span " + " ".join(f"{v:.2f}" for v in r["span"]) +
          " | alone: variant " + " ".join(f"{v:.2f}" for v in r["variant"]) +
          " dense " + " ".join(f"{v:.2f}" for v in r["dense"]) + " rare " + " ".join(f"{v:.2f}" for v in r["rare"]),
          flush=True)
