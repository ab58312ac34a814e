"""Full-size parity and the allocator regression.

* C2 at its bench size (1000 x 2 Mbp, DNA k=21, both strands): the
  complement-sparse words at their real extent (62 K sparse words, so the
  16-bit packed counters run over many chunks) against the CPU oracle, rows
  0, 499 and 998 in full, bit-exact counts and fp64 distances. The oracle
  packs every genome (threads: the C restatement releases the GIL) and
  merges each row set against every column set.
* C3 at its bench size (10,000 x 33,333 aa proteomes, protein k=8, p <= 0.10)
  through METHOD_AUTO, which must pick the two-tier bitsets with a rare tier:
  the bench's whole upper triangle into device outputs (the replayed step),
  rows 0, 4,999 and 9,998 in full against the oracle
  (FastaDistanceProcessor.java:157-186 shape).
* C5 at its bench size (50,000 bottom-1000 sketches of 100 kbp genomes, DNA
  k=21; WidthProcessor.java:178-185): the device sketches of a sample of
  genomes against oracle.sketch, and full rows of the bench's whole-triangle
  sketch matrix against oracle.sketch_distance over every column.
* C4 at its bench size (100,000 x 100 kbp, DNA k=21, p <= 0.05) on one GPU,
  in a subprocess (tests/c4_worker.py): the consuming code all-gather on a
  one-rank RCCL communicator, then rank 0's rows 0-63 and the last rank's
  first rows of the 8-GPU partition against every column; three rows in full
  against the oracle.
* The round-1 fault sequence (a sorted and a bitset workload, then a pack, in
  one process) with its codes checked against the oracle.
"""
import concurrent.futures as cf
import os
import subprocess
import sys

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


def _full_row(M, i):
    """Row i of a square upper-triangle output: (j, i) for j < i, (i, j) for j > i."""
    r = M[i].copy()
    r[:i] = M[:i, i]
    return r


@pytest.mark.timeout(900)
def test_c3_full_size_auto_vs_oracle(ctx, opts):
    """C3 at full size through METHOD_AUTO: the grouped rare tier (round 5,
    the default at this size: the rare kmers as 16-kmer variant words, the
    short-list walk) and the two-tier dictionary with posting lists (option
    rare_group 0); rows 0, 4999 and 9998 in full against the oracle."""
    import gdist
    from gdist import synth
    n, L = 10000, 33_333
    g = synth.genomes(n, L, 0.10, 3, protein=True)           # bench.py's C3 workload (cfg seed 3)
    blob, off = synth.to_blob(g)
    del g
    seqs = [bytes(blob[off[i]:off[i + 1]]) for i in range(n)]
    rows = (0, 4999, 9998)
    with cf.ThreadPoolExecutor(_threads()) as ex:
        row_codes = list(ex.map(lambda i: oracle.kmer_codes(seqs[i], 8, 1, 0), rows))

        def column(j):
            cj = oracle.kmer_codes(seqs[j], 8, 1, 0)
            return [(oracle.intersect(rc, cj), len(cj)) for rc in row_codes]
        cols = list(ex.map(column, range(n)))
    del seqs
    eIs = [np.array([cols[j][r][0] for j in range(n)], np.int64) for r in range(len(rows))]
    eDs = [np.array([oracle.distance(int(eIs[r][j]), len(rc), int(cols[j][r][1])) for j in range(n)])
           for r, rc in enumerate(row_codes)]
    for tier in ("grouped", "two_tier"):
        opts(rare_group=0 if tier == "two_tier" else None)
        sets = gdist.KmerSets.from_blob(blob, off, 8, gdist.KmerType.PROT, 0, ctx)
        chosen, cb, cs = sets.prepare(gdist.METHOD_AUTO)
        assert chosen == gdist.METHOD_BITSET and 0 < cb < cs, (tier, chosen, cb, cs)
        thr, lists, recs = sets.rare_info()
        if tier == "grouped":
            wk, mb, _ = sets.variant_layout()
            assert thr == 2 and lists == 0 and (wk, mb) == (16, 4), (thr, lists, wk, mb)
        else:
            assert thr > 2 and lists > 0 and recs > lists, "C3 must run the two-tier dictionary with a rare tier"
        dI, dD = ctx.alloc(n * n * 4), ctx.alloc(n * n * 8)
        # plan + capture + replay, as the bench steps; the outputs poisoned
        # before every call (a replayed graph that dropped
        # a family's launch would otherwise keep an earlier call's counts),
        # and every call's three rows checked
        pI, pD = np.full(n * n, -7, np.int32), np.full(n * n, 42.5)
        for call in range(3):
            dI.from_host(pI)
            dD.from_host(pD)
            sets.matrix_device(dI.ptr, dD.ptr, n, (0, n), (0, n), upper=True, method=gdist.METHOD_AUTO)
            I = dI.to_host(np.int32).reshape(n, n)
            D = dD.to_host(np.float64).reshape(n, n)
            for r, (i, rc) in enumerate(zip(rows, row_codes)):
                m = np.arange(n) != i
                gi, gd = _full_row(I, i).astype(np.int64), _full_row(D, i)
                assert np.array_equal(gi[m], eIs[r][m]), (tier, call, i, np.flatnonzero((gi != eIs[r]) & m)[:8])
                assert bits_equal(gd[m], eDs[r][m]), (tier, call, i)
            del I, D
        dI.free(); dD.free()
        del sets, pI, pD


@pytest.mark.timeout(900)
def test_c5_full_size_vs_oracle(ctx):
    import gdist
    from gdist import synth
    n, L, w = 50000, 100_000, 1000
    g = synth.genomes(n, L, 0.05, 5)                          # bench.py's C5 workload (cfg seed 5)
    blob, off = synth.to_blob(g)
    del g
    sets = gdist.KmerSets.from_blob(blob, off, 21, gdist.KmerType.DNA, 0, ctx)
    sk = sets.sketches(w)
    del sets
    soff, sigs = sk.download()
    assert len(soff) == n + 1 and np.all(np.diff(soff) == w), "100 kbp genomes hold more than 1000 kmers"
    sig = [sigs[soff[i]:soff[i + 1]] for i in range(n)]
    # the sketches themselves: a sample of genomes against the oracle
    rng = np.random.default_rng(55)
    sample = sorted({0, 24999, 49998, n - 1} | set(rng.choice(n, 300, replace=False).tolist()))

    def oracle_sketch(i):
        return oracle.sketch(oracle.kmer_codes(bytes(blob[off[i]:off[i + 1]]), 21, 0, 0), 21, 0, w)
    with cf.ThreadPoolExecutor(_threads()) as ex:
        osk = list(ex.map(oracle_sketch, sample))
    del blob
    for i, e in zip(sample, osk):
        assert np.array_equal(sig[i], e), i
    # the bench's whole upper triangle into device outputs (plan, replay)
    dC, dD = ctx.alloc(n * n * 4), ctx.alloc(n * n * 8)
    for _ in range(2):
        sk.matrix_device(dC.ptr, dD.ptr, n, (0, n), (0, n), upper=True)
    ctx.synchronize()

    def expect(i):
        e = [oracle.sketch_distance(sig[i], sig[j], w) for j in range(n)]
        return np.array([c for _, c in e], np.int64), np.array([d for d, _ in e])
    for i in (0, 24999):
        eC, eD = expect(i)
        gc = dC.to_host(np.int32, n - i - 1, i * n + i + 1).astype(np.int64)
        gd = dD.to_host(np.float64, n - i - 1, i * n + i + 1)
        assert np.array_equal(gc, eC[i + 1:]), (i, np.flatnonzero(gc != eC[i + 1:])[:8])
        assert bits_equal(gd, eD[i + 1:]), i
        # and 2,000 random pairs of the triangle
    pairs = [(int(a), int(b)) for a, b in rng.integers(0, n, (4000, 2)) if a < b][:2000]
    for a, b in pairs:
        d, c = oracle.sketch_distance(sig[a], sig[b], w)
        assert int(dC.to_host(np.int32, 1, a * n + b)[0]) == c and bits_equal(dD.to_host(np.float64, 1, a * n + b), [d])
    dC.free(); dD.free()
    # full rows (both sides of the diagonal) through a row-block call
    for i in (24999, 49998):
        C, Dr = sk.matrix((i, i + 1), (0, n))
        eC, eD = expect(i)
        assert np.array_equal(C[0].astype(np.int64), eC) and bits_equal(Dr[0], eD), i


def test_pack_after_bitset_workload_regression(ctx):
    """The sequence that produced wrong codes under the stream-ordered pool
    (round 1's diag_pack.py diagnostic): sorted and bitset matrix workloads, then a
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


@pytest.mark.timeout(1150)
def test_c4_full_size_slices_vs_oracle():
    """C4 (BASELINE configs[3]) at its size: see tests/c4_worker.py."""
    import gc

    import gdist
    # the worker needs most of the GPU: this process's cached device blocks
    # (the full-size tests above freed tens of GB into the library's cache)
    # go back to the driver first
    gc.collect()
    gdist.release_device_cache(0)
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "c4_worker.py")], capture_output=True, text=True,
                       timeout=1100)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "C4_OK" in r.stdout
