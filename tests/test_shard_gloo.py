"""CPU, world size 2 over gloo: the row-sharded N×N decomposition used by
bench.py / SURVEY §8e reproduces the unsharded upper triangle. Each rank
packs its own shard of genomes, the shards are all-gathered (gloo stands in
for the RCCL all-gather here), and each rank computes its equal-area row
block; the blocks merged on rank 0 equal the single-process result."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    for p in (os.path.join(ROOT, "genome.distance_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import oracle
    from gdist import shard, synth
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s0, s1 = shard.shard_of_sets(n, world)[rank]
    g = synth.genomes(s1 - s0, 3000, 0.05, 7, first=s0)
    off, codes = oracle.pack([bytes(r) for r in g], 13)
    shards = [None] * world
    dist.all_gather_object(shards, (off, codes))           # the packed-set all-gather
    all_off = [0]
    all_codes = []
    for o, c in shards:
        for x in np.diff(o):
            all_off.append(all_off[-1] + int(x))
        all_codes.append(c)
    all_off = np.array(all_off, np.int64)
    all_codes = np.concatenate(all_codes)
    b = shard.triangle_bounds(n, world, 8)
    r0, r1 = b[rank], b[rank + 1]
    _, D = oracle.matrix(all_off, all_codes, r0, r1, 0, n, flags=0x100)
    blocks = [None] * world
    dist.all_gather_object(blocks, (r0, r1, D))
    if rank == 0:
        q.put(shard.merge_row_blocks(blocks, n))
    dist.barrier()
    dist.destroy_process_group()


def test_row_sharded_triangle_matches_unsharded():
    pytest.importorskip("torch.distributed")
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from gdist import shard, synth
    n, world = 37, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    merged = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = synth.genomes(n, 3000, 0.05, 7)
    off, codes = oracle.pack([bytes(r) for r in g], 13)
    _, D = oracle.matrix(off, codes, 0, n, 0, n, flags=0x100)
    iu = np.triu_indices(n, 1)
    assert np.array_equal(merged[iu].view(np.uint64), D[iu].view(np.uint64))
    # every pair is owned by exactly one rank
    b = shard.triangle_bounds(n, world, 8)
    assert sum(shard.pairs_in_rows(n, b[r], b[r + 1]) for r in range(world)) == n * (n - 1) // 2


def test_synth_shards_equal_whole():
    from gdist import shard, synth
    whole = synth.genomes(10, 500, 0.1, 3)
    parts = [synth.genomes(b - a, 500, 0.1, 3, first=a) for a, b in shard.shard_of_sets(10, 3)]
    assert np.array_equal(np.concatenate(parts), whole)


def test_balanced_bounds():
    """Min-max modelled time per rank: dense (area) + per-row costs, and a
    cost with a fixed per-block term (list-major rare tier)."""
    from gdist import shard
    for n, G in ((1000, 2), (2000, 4), (2828, 8), (50, 8), (7, 3)):
        tot = n * (n - 1) / 2
        for dense, row, fixed in ((1.0, 0.0, 0.0), (1.0, 0.5, 0.0), (0.2, 1.0, 0.0), (0.0, 1.0, 0.0),
                                  (1.0, 0.3, 0.05)):
            def cost(r0, r1):
                if r1 <= r0:
                    return 0.0
                return dense * shard.pairs_in_rows(n, r0, r1) / tot + row * (r1 - r0) / n + fixed
            b = shard.balanced_bounds(n, G, cost)
            assert len(b) == G + 1 and b[0] == 0 and b[-1] == n and all(x <= y for x, y in zip(b, b[1:]))
            costs = [cost(b[g], b[g + 1]) for g in range(G)]
            step = dense * (n - 1) / tot + row / n            # the most one row can add
            assert max(costs) <= sum(costs) / G + step + 1e-9, (n, G, dense, row, b)
            if (row, fixed) == (0.0, 0.0):                   # pure area: the equal-area partition
                eq = shard.triangle_bounds(n, G, 1)
                assert all(abs(x - y) <= 1 for x, y in zip(b, eq)), (b, eq)
            # no partition has a smaller maximum than one more row can explain
            eq_area = [cost(x, y) for x, y in zip(shard.triangle_bounds(n, G, 1), shard.triangle_bounds(n, G, 1)[1:])]
            assert max(costs) <= max(eq_area) + 1e-9