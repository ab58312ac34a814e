"""In-process A/B of context options (gdist_ctx_set_option, named GDIST_<OPTION> here):
interleaved rounds on one collection; every setting's counts must equal the
first one's. AB_ENVS="K=V,K=V;K=V;..." (";" separates settings, "" = defaults),
AB_N sets (C2-like 2 Mbp genomes; AB_CONFIG=c2r: C2-realistic), AB_BLOCKS="r0:r1 ..." row blocks (default
the whole triangle), or AB_RANKS=G: the G blocks of the cost-balanced partition."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import shard, synth

n = int(os.environ.get("AB_N", "1000"))
settings = [s for s in os.environ.get("AB_ENVS", "").split(";")]
rounds = int(os.environ.get("AB_ROUNDS", "5"))
ctx = gdist.Context(0)
ctx.set_option("step_timing", 1)     # graph-replayed steps record their kernel times too
if os.environ.get("AB_CONFIG", "c2") == "c2r":       # C2-realistic (bench.py CONFIGS["c2r"])
    seqs = synth.realistic_genomes(n, 2_000_000, 0.002, 2)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    del seqs
else:
    g = synth.genomes(n, 2_000_000, 0.002, 2)
    blob, off = synth.to_blob(g); del g
    sets = gdist.KmerSets.from_sequences([blob[off[i]:off[i + 1]] for i in range(n)], 21, gdist.KmerType.DNA, 0, ctx)
    del blob
sets.build_bitsets()
blocks = []
for b in os.environ.get("AB_BLOCKS", f"0:{n}").split():
    a, c = (int(x) for x in b.split(":"))
    blocks.append((a, c))
if os.environ.get("AB_RANKS"):
    G = int(os.environ["AB_RANKS"])
    bd = shard.balanced_bounds(n, G, lambda a, c: sets.block_cost((a, c))[0])
    blocks = [(bd[r], bd[r + 1]) for r in range(G)]
rows = max(c - a for a, c in blocks)
dI, dD = ctx.alloc(rows * n * 4), ctx.alloc(rows * n * 8)
print(f"n={n} blocks={blocks}", flush=True)
def opt_name(kv):
    return kv[len("GDIST_"):].lower() if kv.startswith("GDIST_") else kv.lower()


base = {}
for kv in set(k for s in settings for k in [x.split("=")[0] for x in s.split(",") if x]):
    base[kv] = ctx.option(opt_name(kv))
times = {s: {b: [] for b in blocks} for s in settings}
ref = {}
for rnd in range(rounds):
    for s in settings:
        for kv, v in base.items():
            ctx.set_option(opt_name(kv), v)
        for x in s.split(","):
            if x:
                kk, vv = x.split("=")
                ctx.set_option(opt_name(kk), int(vv))
        for b in blocks:
            sets.matrix_device(dI.ptr, dD.ptr, n, b, (0, n), upper=True, method=gdist.METHOD_BITSET)
            ctx.synchronize()
            times[s][b].append(ctx.last_timing()[0])
            if rnd == 0:
                I = dI.to_host(np.int32, (b[1] - b[0]) * n).reshape(b[1] - b[0], n)
                up = np.fromfunction(lambda i, j: j > i + b[0], I.shape)
                if b not in ref:
                    ref[b] = I[up].copy()
                else:
                    assert np.array_equal(ref[b], I[up]), (s, b)
for s in settings:
    med = [float(np.median(times[s][b][1:] or times[s][b])) for b in blocks]
    print(f"[{s or 'default'}] kernel ms per block {[round(x, 3) for x in med]} max {max(med):.3f} sum {sum(med):.3f}",
          flush=True)
