"""In-process A/B on C3 (bench.py --config c3, or AB_CONFIG=c3r): the
collection built once with METHOD_AUTO, then per setting (AB_ENVS="k=v,k=v;..."
of context options, "" = defaults) interleaved rounds of the full upper
triangle: the step's kernel span (graph-replayed) and, with serial_step = 1
and time_kernels = 1, each kernel family alone (dense tiles, variant / rare
walk). Every setting's counts must equal the first one's."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import synth

N, L, P, CFG, K = 10_000, 33_333, 0.10, 3, 8
settings = os.environ.get("AB_ENVS", "").split(";")
rounds = int(os.environ.get("AB_ROUNDS", "3"))
t0 = time.time()
ctx = gdist.Context(0)
if os.environ.get("AB_CONFIG", "c3") == "c3r":
    seqs = synth.realistic_genomes(N, L, P, CFG, protein=True)
else:
    g = synth.genomes(N, L, P, CFG, protein=True)
    blob, off = synth.to_blob(g)
    del g
    seqs = [blob[off[i]:off[i + 1]] for i in range(N)]
sets = gdist.KmerSets.from_sequences(seqs, K, gdist.KmerType.PROT, 0, ctx)
del seqs
chosen, _, _ = sets.prepare(gdist.METHOD_AUTO, pairs=float(N * (N - 1) // 2))
assert chosen == gdist.METHOD_BITSET, chosen
print(f"built in {time.time() - t0:.1f} s", flush=True)
dI, dD = ctx.alloc(N * N * 4), ctx.alloc(N * N * 8)
up = np.fromfunction(lambda i, j: j > i, (N, N))
ref = None
fams = ("dense", "variant", "rare")
res = {s: {"span": [], **{f: [] for f in fams}} for s in settings}
names = sorted({kv.split("=")[0] for s in settings for kv in s.split(",") if kv})
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
        for _ in range(3):
            sets.matrix_device(dI.ptr, dD.ptr, N, (0, N), (0, N), upper=True, method=gdist.METHOD_BITSET)
        ctx.synchronize()
        res[s]["span"].append(ctx.last_timing()[0])
        ctx.set_option("time_kernels", 1)
        ctx.set_option("serial_step", 1)
        sets.matrix_device(dI.ptr, dD.ptr, N, (0, N), (0, N), upper=True, method=gdist.METHOD_BITSET)
        ctx.synchronize()
        for f in fams:
            res[s][f].append(ctx.kernel_ms(f))
        ctx.set_option("time_kernels", None)
        ctx.set_option("serial_step", None)
        if rnd == 0 and "variant_short=9" not in s:     # 9: the walk without its flush (timing only)
            I = dI.to_host(np.int32, N * N).reshape(N, N)[up]
            if ref is None:
                ref = I.copy()
            else:
                assert np.array_equal(I, ref), f"setting {s!r}: counts differ"
for s in settings:
    r = res[s]
    print(f"[{s or 'default'}] span " + " ".join(f"{v:.3f}" for v in r["span"]) + " | alone: " +
          " ".join(f"{f} " + " ".join(f"{v:.3f}" for v in r[f]) for f in fams), flush=True)
