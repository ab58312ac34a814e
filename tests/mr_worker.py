"""Worker of tests/test_multirank_gpu.py, one process per rank (launched by
torch.distributed.run, gloo): the row-sharded multi-rank path on ranks that
share one GPU through the host-staged transport. For every case each rank
packs its shard, all-gathers (bitsets, plain sets, sketches), computes its
triangle rows, and rank 0 compares every rank's rows bit-exactly with the CPU
oracle over all sets.

Cases:
  base    301 x 6 kbp, p 0.01: bitset, sorted and sketch (C5's exchange) legs
  sparse  C2-shaped (shared core, p <= 0.002): the complement-sparse words
          must be active on every rank, so the rank-tagged locus keys are
          all-gathered and min-reduced (gdist_sets_allgather_bitsets)
  c4      C4-shaped (100 kbp, p <= 0.05, DNA k=21) at small N, METHOD_AUTO,
          and the exchange plan under a memory budget too small for the
          dictionary exchange: the in-place code all-gather that consumes the
          local shard (what C4 at 100,000 genomes on 8 GPUs runs)
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gdist  # noqa: E402
import oracle  # noqa: E402  (test infrastructure: the checker)
from gdist import shard, synth  # noqa: E402

CASES = {
    "base": dict(n=301, L=6000, p=0.01, cfg=11, legs=("bitset", "sorted", "sketch", "reps")),
    "sparse": dict(n=300, L=150_000, p=0.002, cfg=12, legs=("bitset",), sparse=True),
    "c4": dict(n=200, L=100_000, p=0.05, cfg=4,
               legs=("auto", "auto_gathered", "sorted", "codes_plan", "codes_variant", "codes_two_tier")),
}
SKETCH_W = 200
REPS_T = 0.35


def run_case(name, c, ctx, rank, world):
    n = c["n"]
    seqs = [bytes(r) for r in synth.genomes(n, c["L"], c["p"], c["cfg"])]
    s0, s1 = shard.shard_of_sets(n, world)[rank]
    local = gdist.KmerSets.from_sequences(seqs[s0:s1], 21, gdist.KmerType.DNA, 0, ctx)
    bounds = shard.triangle_bounds(n, world, 16)
    r0, r1 = bounds[rank], bounds[rank + 1]
    results = {}
    info = {}
    for leg in c["legs"]:
        if leg in ("bitset", "auto"):
            gb = local.allgather_bitsets()
            assert len(gb) == n
            if c.get("sparse"):
                ws, wd, ent = gb.sparse_info()
                assert ws > 0 and ent > 0, f"rank {rank}: complement-sparse words not active"
                info["sparse"] = (ws, wd, ent)
            results[leg] = gb.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
        elif leg == "sorted":
            gs = local.allgather()
            assert len(gs) == n
            results[leg] = gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_SORTED)
        elif leg == "auto_gathered":
            # METHOD_AUTO on a replicated code collection: its build
            # is collective, and each rank prices its own region, so rank 0
            # asks for the whole triangle and the others for a handful of
            # pairs — the per-rank estimates disagree, the keep/free verdict
            # must not. Called twice: a rank left without the bits would enter
            # the next collective build alone (a hang, not a wrong count).
            gs = local.allgather()
            pairs = 0.5 * n * (n - 1) if rank == 0 else float(rank)
            m1, _, _ = gs.prepare(gdist.METHOD_AUTO, pairs)
            m2, _, _ = gs.prepare(gdist.METHOD_AUTO, pairs)
            info["auto_methods"] = (m1, m2)
            results[leg] = gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_AUTO)
            I2, D2 = gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_AUTO)
            assert np.array_equal(I2, results[leg][0]), rank
            # a BITSET call after AUTO: the collective build (if AUTO freed the
            # bits) is entered by every rank or by none
            results["auto_then_bitset"] = gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
        elif leg == "codes_plan":
            m, bb, bc = local.exchange_plan()
            assert m == gdist.METHOD_BITSET, (m, bb, bc)            # small: the dictionary exchange fits
            budget = 1 << 30
            assert bc <= budget < bb, (bb, bc)
            # the bitsets estimate counts the bitsets the exchange allocates: at
            # least every set's ancestral words (~200 K kmers both strands)
            assert bb >= n * (200_000 // 64) * 8, bb
            ctx.set_option("exchange_budget", budget)
            own = gdist.KmerSets.from_sequences(seqs[s0:s1], 21, gdist.KmerType.DNA, 0, ctx)
            m, _, _ = own.exchange_plan()
            assert m == gdist.METHOD_SORTED, m
            gs = own.allgather(consume=True)
            ctx.set_option("exchange_budget", None)
            assert len(gs) == n and len(own) == s1 - s0
            # a consumed shard holds neither codes nor bitsets: every method and
            # the greedy reps refuse it (EINVAL) instead of reading released memory
            for call in (lambda: own.matrix(method=gdist.METHOD_SORTED),
                         lambda: own.matrix(method=gdist.METHOD_BITSET),
                         lambda: own.matrix(method=gdist.METHOD_AUTO),
                         lambda: own.greedy_reps(0.5)):
                try:
                    call()
                    raise AssertionError("a consumed shard must refuse distance calls")
                except ValueError:
                    pass
            results[leg] = gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_SORTED)
        elif leg == "codes_variant":
            # C4's 8-GPU path: the consuming code all-gather, then on every rank
            # the dictionary tiers of the gathered codes with the variant tier
            # (forced at this size: kmers of 2..19 sets are variant words),
            # located by rank 0's guides that travel with the gather
            own = gdist.KmerSets.from_sequences(seqs[s0:s1], 21, gdist.KmerType.DNA, 0, ctx)
            gs = own.allgather(consume=True)
            for k, v in (("variant", 1), ("rare_t", 2), ("variant_dmin", 20), ("range_summary", 1)):
                ctx.set_option(k, v)
            m, _, _ = gs.prepare(gdist.METHOD_BITSET)
            vk, vw, ve, _ = gs.variant_info()
            assert vk > 0 and ve > 0 and vw * 4 < vk, (rank, vk, vw, ve)
            info["variant"] = (vk, vw, ve)
            # round 5: the gathered collection's build is split by rank (each
            # rank 1/R of the code ranges and of the sets' fill, the tiers
            # all-gathered), then the codes are released
            bt = gs.build_timing()
            assert bt["shares"] == world, (rank, bt)
            gs.release_codes()
            results[leg] = gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
            try:
                gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_SORTED)
                raise AssertionError("released codes must refuse the sorted join")
            except ValueError:
                pass
            for k in ("variant", "rare_t", "variant_dmin", "range_summary"):
                ctx.set_option(k, None)
        elif leg == "codes_two_tier":
            # the two-tier build of a gathered collection, split by rank (the
            # windowed fill of each rank's sets, rows and rare records gathered)
            own = gdist.KmerSets.from_sequences(seqs[s0:s1], 21, gdist.KmerType.DNA, 0, ctx)
            gs = own.allgather(consume=True)
            for k, v in (("variant", 0), ("rare_t", 3)):
                ctx.set_option(k, v)
            gs.build_bitsets()
            assert gs.variant_info()[0] == 0 and gs.rare_info()[1] > 0, (rank, gs.rare_info())
            assert gs.build_timing()["shares"] == world
            results[leg] = gs.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
            for k in ("variant", "rare_t"):
                ctx.set_option(k, None)
        elif leg == "reps":
            # greedy representatives of a gathered collection:
            # every rank computes each block against its 1/R of the columns,
            # cover flags and closest representatives combined by all-gathers
            gs = local.allgather()
            ctx.set_option("reps_block", 100)                   # four blocks of rows
            is_rep, rep_of, rep_d = gs.greedy_reps(REPS_T, assign=True, method=gdist.METHOD_BITSET)
            ctx.set_option("reps_block", None)
            info["reps"] = (is_rep.tolist(), rep_of.tolist(), rep_d.tolist())
            continue
        elif leg == "sketch":
            sk = local.sketches(SKETCH_W).allgather()
            assert len(sk) == n
            so, sv = sk.download()
            results[leg] = sk.matrix((r0, r1), (0, n), upper=True)
            info["sketch_sigs"] = [sv[so[i]:so[i + 1]].tolist() for i in range(n)]
    gathered = [None] * world
    dist.all_gather_object(gathered, (r0, r1, {m: (I.tolist(), D.tolist()) for m, (I, D) in results.items()},
                                      info))
    if rank != 0:
        return
    off, codes = oracle.pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n, flags=0x100, nthreads=8)
    esk = [oracle.sketch(codes[off[i]:off[i + 1]], 21, 0, SKETCH_W) for i in range(n)] \
        if "sketch" in c["legs"] else None
    if "reps" in c["legs"]:
        # every rank the same answer, equal to the greedy pass over the oracle's distances
        first = gathered[0][3]["reps"]
        assert all(g[3]["reps"] == first for g in gathered), (name, "ranks disagree on the representatives")
        is_rep, rep_of, rep_d = first
        sD = np.triu(eD, 1) + np.triu(eD, 1).T          # eD holds the upper triangle only
        reps = []
        for i in range(n):
            if not any(sD[i, r] <= REPS_T for r in reps):
                reps.append(i)
        assert [i for i in range(n) if is_rep[i]] == reps, (name, "representatives")
        for i in range(n):
            if not is_rep[i]:
                cand = [(sD[i, r], r) for r in reps if sD[i, r] < 1.0]
                best = min(cand) if cand else (1.0, -1)
                assert rep_d[i] == best[0] and rep_of[i] == best[1], (name, i, rep_of[i], rep_d[i], best)
    if "auto_gathered" in c["legs"]:
        am = [g[3]["auto_methods"] for g in gathered]
        assert all(x == am[0] and x[0] == x[1] for x in am), (name, "ranks disagree on AUTO's method", am)
    rows = 0
    for (a, b, res, inf) in gathered:
        up = np.fromfunction(lambda x, y: y > (a + x), (b - a, n))
        for m, (I, D) in res.items():
            I, D = np.array(I, dtype=np.int32), np.array(D, dtype=np.float64)
            if m == "sketch":
                assert inf["sketch_sigs"] == [s.tolist() for s in esk], (name, "sketch signatures")
                for i in range(a, b):
                    for j in range(i + 1, n):
                        d, common = oracle.sketch_distance(esk[i], esk[j], SKETCH_W)
                        assert I[i - a, j] == common and D[i - a, j] == d, (name, m, i, j)
                continue
            assert np.array_equal(I[up], eI[a:b][up]), (name, m, a, b)
            assert np.array_equal(D[up].view(np.uint64), eD[a:b][up].view(np.uint64)), (name, m, a, b)
        rows += b - a
    assert rows == n
    print(f"CASE_OK {name} {world} {gathered[0][3].get('sparse', '')} {gathered[0][3].get('variant', '')}", flush=True)


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ctx = gdist.Context(0)

    def ag(a):
        t = torch.from_numpy(a)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return torch.cat(outs).numpy()

    ctx.comm_init_host(world, rank, ag)
    assert ctx.allreduce_max(float(rank)) == float(world - 1)
    names = os.environ.get("MR_CASES", ",".join(CASES)).split(",")
    for name in names:
        run_case(name, CASES[name], ctx, rank, world)
        dist.barrier()
    if rank == 0:
        print("MULTIRANK_OK", world, flush=True)
    ctx.comm_destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
