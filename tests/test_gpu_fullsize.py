"""Full-size parity and the allocator regression.

* C2 at its bench size (1000 x 2 Mbp, DNA k=21, both strands): the
  complement-sparse words at their real extent (62 K sparse words, so the
  16-bit packed counters run over many chunks) against the CPU oracle, rows
  0, 499 and 998 in full, bit-exact counts and fp64 distances. The oracle
  packs every genome (threads: the C restatement releases the GIL) and
  merges each row set against every column set.
* The round-1 fault sequence (a sorted and a bitset workload, then a pack, in
  one process) with its codes checked against the oracle.
"""
import concurrent.futures as cf
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64))


def _threads():
    omp = os.environ.get("OMP_NUM_THREADS", "")
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return max(1, min(aff, int(omp))) if omp.isdigit() and int(omp) > 0 else max(1, min(aff, 16))


@pytest.mark.timeout(900)
def test_c2_full_size_rows_vs_oracle(ctx, opts):
    import gdist
    from gdist import synth
    n, L = 1000, 2_000_000
    g = synth.genomes(n, L, 0.002, 2)                # bench.py's C2 workload (cfg seed 2)
    blob, off = synth.to_blob(g)
    del g
    seqs = [bytes(blob[off[i]:off[i + 1]]) for i in range(n)]
    del blob
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    ws, wd, ent = sets.sparse_info()
    assert ws > 1023 and ent > 0, "C2 must run the complement-sparse words over several 16-bit counter chunks"
    I, D = sets.matrix(upper=False, method=gdist.METHOD_BITSET)
    rows = (0, 499, 998)
    with cf.ThreadPoolExecutor(_threads()) as ex:
        row_codes = list(ex.map(lambda i: oracle.kmer_codes(seqs[i], 21, 0, 0), rows))

        def column(j):
            cj = oracle.kmer_codes(seqs[j], 21, 0, 0)
            return [(oracle.intersect(rc, cj), len(cj)) for rc in row_codes]
        cols = list(ex.map(column, range(n)))
    for r, (i, rc) in enumerate(zip(rows, row_codes)):
        eI = np.array([cols[j][r][0] for j in range(n)], np.int64)
        nb = np.array([cols[j][r][1] for j in range(n)], np.int64)
        eD = np.array([oracle.distance(int(eI[j]), len(rc), int(nb[j])) for j in range(n)])
        assert np.array_equal(I[i].astype(np.int64), eI), (i, np.flatnonzero(I[i] != eI)[:8])
        assert bits_equal(D[i], eD), i
    # the whole triangle is symmetric (rows and columns of one pair agree)
    assert np.array_equal(I, I.T)
    # the default pack keeps its four chunks' summaries for the dictionary; the
    # set-major pack (option pack_summary 0) leaves the bitset build to sort
    # every code: the same dictionary, sparse plan and counts
    info = (sets.build_bitsets(), sets.sparse_info())
    del sets
    opts(pack_summary=0)
    s0 = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    assert (s0.build_bitsets(), s0.sparse_info()) == info
    I0, _ = s0.matrix((0, 200), (0, n), upper=False, method=gdist.METHOD_BITSET)
    assert np.array_equal(I0, I[:200])


def test_pack_after_bitset_workload_regression(ctx):
    """The sequence that produced wrong codes under the stream-ordered pool
    (scripts/diag/diag_pack.py): sorted and bitset matrix workloads, then a
    pack of another collection, in one process and on one context. Codes,
    sizes and a matrix of the fresh pack equal the oracle on every trial."""
    import gdist
    from gdist import synth
    seqs = [bytes(r) for r in synth.genomes(300, 3000, 0.05, 91)]
    s2 = [bytes(r) for r in synth.genomes(150, 5000, 0.01, 92)]
    off, codes = oracle.pack(s2, 21)
    eI, _ = oracle.matrix(off, codes, 0, 150, 0, 150)
    for trial in range(4):
        for method in (gdist.METHOD_SORTED, gdist.METHOD_BITSET):
            w = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
            if method == gdist.METHOD_BITSET:
                w.build_bitsets()
            w.matrix(method=method)
            del w
        a = gdist.KmerSets.from_sequences(s2, 21, gdist.KmerType.DNA, 0, ctx)
        oa, ca = a.download()
        assert np.array_equal(oa, off) and np.array_equal(ca, codes), trial
        a.build_bitsets()
        Ia, _ = a.matrix(method=gdist.METHOD_BITSET)
        assert np.array_equal(Ia, eI), trial
        del a
