"""Worker of tests/test_multirank_gpu.py, one process per rank (launched by
torch.distributed.run, gloo): the row-sharded multi-rank path on ranks that
share one GPU through the host-staged transport. Each rank packs its shard,
all-gathers (bitsets and plain sets), computes its triangle rows, and rank 0
compares every rank's rows with a single-process matrix over all sets."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import gdist  # noqa: E402
from gdist import shard, synth  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    n, L = int(os.environ.get("MR_N", "301")), int(os.environ.get("MR_LEN", "6000"))
    ctx = gdist.Context(0)

    def ag(a):
        t = torch.from_numpy(a)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return torch.cat(outs).numpy()

    ctx.comm_init_host(world, rank, ag)
    assert ctx.allreduce_max(float(rank)) == float(world - 1)
    g = synth.genomes(n, L, 0.01, 11)
    seqs = [bytes(r) for r in g]
    s0, s1 = shard.shard_of_sets(n, world)[rank]
    local = gdist.KmerSets.from_sequences(seqs[s0:s1], 21, gdist.KmerType.DNA, 0, ctx)
    bounds = shard.triangle_bounds(n, world, 16)
    r0, r1 = bounds[rank], bounds[rank + 1]
    results = {}
    gb = local.allgather_bitsets()
    assert len(gb) == n
    results["bitset"] = gb.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
    gs = local.allgather()
    assert len(gs) == n and np.array_equal(gs.sizes(), gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx).sizes())
    results["sorted"] = gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_SORTED)
    gathered = [None] * world
    dist.all_gather_object(gathered, (r0, r1, {m: (I.tolist(), D.tolist()) for m, (I, D) in results.items()}))
    if rank == 0:
        full = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
        eI, eD = full.matrix(upper=True, method=gdist.METHOD_SORTED)
        rows = 0
        for (a, b, res) in gathered:
            up = np.fromfunction(lambda x, y: y > (a + x), (b - a, n))
            for m, (I, D) in res.items():
                I, D = np.array(I, dtype=np.int32), np.array(D, dtype=np.float64)
                assert np.array_equal(I[up], eI[a:b][up]), (m, a, b)
                assert np.array_equal(D[up].view(np.uint64), eD[a:b][up].view(np.uint64)), (m, a, b)
            rows += b - a
        assert rows == n
        print("MULTIRANK_OK", world, flush=True)
    ctx.comm_destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
