"""Worker of tests/test_gpu_fullsize.py::test_c4_full_size_slices_vs_oracle:
C4 at its bench size on one GPU, in its own process (RCCL communicator, the
160 GB of gathered codes released at exit).

C4 = 100,000 synthetic 100 kbp genomes, DNA k=21 both strands, p <= 0.05,
cfg seed 4 (bench.py CONFIGS["c4"]). On the 8-GPU node every rank packs its
shard and ONE in-place code all-gather gives every rank all 100,000 sets
(DESIGN.md §6); here one GPU holds the whole collection, packed from one host
buffer, and the same consuming all-gather runs through ncclAllGather on a
one-rank communicator (the path `bench.py --config c4 --rows A:B
--force-exchange` takes). Then the per-rank slices the bench times: rank 0's
rows 0-63 and the first rows of the last rank's block
(gdist.shard.triangle_bounds(100000, 8)), each against every column
(FastaDistanceProcessor.java:157-186: the pair loop of a row block).

Checked against the CPU oracle (the checker): rows 0, 63 and the last
block's first row in full — oracle.kmer_codes of every genome, threaded,
intersected with the three row sets — bit-exact counts and fp64 distances.
Progress lines go to stdout and to gpurun_out/c4_worker.log (a long run that
keeps writing is not taken for a hung one).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gdist  # noqa: E402
import oracle  # noqa: E402  (test infrastructure: the checker)
from gdist import shard, synth  # noqa: E402

N, L, P, CFG, K = 100_000, 100_000, 0.05, 4, 21
T0 = time.time()
LOG = os.path.join(ROOT, "gpurun_out", "c4_worker.log")


def log(msg):
    line = f"[c4 {time.time() - T0:7.1f}s] {msg}"
    print(line, flush=True)
    try:
        os.makedirs(os.path.dirname(LOG), exist_ok=True)
        with open(LOG, "a") as f:
            f.write(line + "\n")
    except OSError:
        pass


def threads():
    omp = os.environ.get("OMP_NUM_THREADS", "")
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return max(1, min(aff, int(omp))) if omp.isdigit() and int(omp) > 0 else max(1, min(aff, 16))


def main():
    ctx = gdist.Context(0)
    ctx.comm_init(gdist.Context.unique_id(), 1, 0)
    g = synth.genomes(N, L, P, CFG)
    blob, off = synth.to_blob(g)
    del g
    log(f"generated {N} x {L} bp")
    local = gdist.KmerSets.from_blob(blob, off, K, gdist.KmerType.DNA, 0, ctx)
    sizes = local.sizes()
    log(f"packed: {int(sizes.sum())} codes")
    m, bb, bc = local.exchange_plan()
    assert m == gdist.METHOD_SORTED, ("C4 must take the code all-gather", m, bb, bc)
    gs = local.allgather(consume=True)
    assert len(gs) == N and np.array_equal(gs.sizes(), sizes)
    log(f"consuming code all-gather done (estimates: bitsets {bb:.3g} B, codes {bc:.3g} B per rank)")
    bounds = shard.triangle_bounds(N, 8, 1)
    last = bounds[7]
    # METHOD_AUTO on the gathered codes, priced on rank 0's block (what the
    # 8-GPU bench asks): the dictionary tiers built from the gathered codes
    # by code ranges — dense ancestral words, the variant tier of the
    # single-substitution kmers, rare posting lists — against the sorted join
    t = time.time()
    chosen, cb, cs = gs.prepare(gdist.METHOD_AUTO, pairs=float(shard.pairs_in_rows(N, bounds[0], bounds[1])))
    vk, vw, ve, vp = gs.variant_info()
    log(f"METHOD_AUTO: {'bitset' if chosen == gdist.METHOD_BITSET else 'sorted'} (est. bitset {cb:.3g} s, "
        f"sorted {cs:.3g} s, {time.time() - t:.1f} s to build); dense words {gs.bitset_info()[1]}, variant tier "
        f"{vk} kmers in {vw} words, {ve} entries, {vp:.3g} products; rare {gs.rare_info()}")
    assert chosen == gdist.METHOD_BITSET and vk > 1_000_000, "C4 takes the variant tier"
    slices = [(0, 64), (last, last + 16)]
    rows = {0: None, 63: None, last: None}
    for method, name in ((gdist.METHOD_BITSET, "bitset+variant"), (gdist.METHOD_SORTED, "sorted join")):
        for (a, b) in slices:
            t = time.time()
            I, D = gs.matrix((a, b), (0, N), upper=True, method=method)
            log(f"{name}: slice rows [{a}, {b}) x {N} columns: {time.time() - t:.2f} s")
            for i in rows:
                if a <= i < b:
                    if rows[i] is None:
                        rows[i] = (I[i - a].copy(), D[i - a].copy())
                    else:                            # both methods: the same bits
                        js = np.arange(i + 1, N)
                        assert np.array_equal(rows[i][0][js], I[i - a][js]), (name, i)
                        assert np.array_equal(rows[i][1][js].view(np.uint64), D[i - a][js].view(np.uint64)), (name, i)
            del I, D
    # the oracle: every genome's codes, intersected with the three row sets
    row_ids = sorted(rows)
    row_codes = [oracle.kmer_codes(bytes(blob[off[i]:off[i + 1]]), K, 0, 0) for i in row_ids]
    assert [len(c) for c in row_codes] == [int(sizes[i]) for i in row_ids]

    # every column's codes extracted and intersected in the oracle's C loop
    # (threaded over columns), 10,000 columns a call so that progress shows
    eI = np.zeros((len(row_ids), N), np.int64)
    nb = np.zeros(N, np.int64)
    for j0 in range(0, N, 10_000):
        j1 = min(N, j0 + 10_000)
        part, sz = oracle.rows_vs_columns(blob[off[j0]:off[j1]], off[j0:j1 + 1] - off[j0], row_codes, K, 0, 0,
                                          nthreads=threads())
        eI[:, j0:j1] = part
        nb[j0:j1] = sz
        log(f"oracle columns {j1} / {N}")
    assert np.array_equal(nb, sizes)
    for r, i in enumerate(row_ids):
        I, D = rows[i]
        js = np.arange(i + 1, N)
        assert np.array_equal(I[js].astype(np.int64), eI[r, js]), (i, js[I[js] != eI[r, js]][:8])
        eD = np.array([oracle.distance(int(eI[r, j]), len(row_codes[r]), int(nb[j])) for j in js])
        assert np.array_equal(D[js].view(np.uint64), eD.view(np.uint64)), i
        log(f"row {i}: {len(js)} pairs bit-exact")
    ctx.comm_destroy()
    print("C4_OK", flush=True)


if __name__ == "__main__":
    main()
