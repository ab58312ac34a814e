"""GPU parity: the HIP path (through libgdist.so's C-ABI) against the CPU
oracle and the committed golden vectors. Bit-exact for codes, counts and
distances (fp64, no tolerance). Parity is unpinned against the reference
itself — these pin the device to the two restatements."""
import io
import json
import math
import os
import random

import numpy as np
import pytest

import oracle
import pyref

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kmer_golden.json")


def golden_cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64))


def oracle_pack(seqs, k, kind, flags):
    return oracle.pack([s if isinstance(s, bytes) else s.encode("latin-1") for s in seqs], k, kind, flags)


# ---------------------------------------------------------------- golden
@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["name"])
def test_golden_through_device(ctx, case):
    import gdist
    kt = gdist.KmerType.DNA if case["kind"] == 0 else gdist.KmerType.PROT
    sets = gdist.KmerSets.from_sequences(case["seqs"], case["k"], kt, case["flags"], ctx)
    off, codes = sets.download()
    got = [[str(int(x)) for x in codes[off[i]:off[i + 1]]] for i in range(len(off) - 1)]
    assert got == case["codes"]
    assert sets.sizes().tolist() == case["sizes"]
    for method in (gdist.METHOD_SORTED, gdist.METHOD_BITSET):
        I, D = sets.matrix(method=method)
        assert I.tolist() == case["I"], method
        assert [[gdist.java_double(x) for x in r] for r in D] == case["D"], method
    w = case["width"]
    sk = sets.sketches(w)
    so, sv = sk.download()
    assert [sv[so[i]:so[i + 1]].tolist() for i in range(len(so) - 1)] == case["sketch"]
    _, SD = sk.matrix()
    assert [[gdist.java_double(x) for x in r] for r in SD] == case["sketch_D"]
    _, SJ = sk.matrix(flags=gdist.SKETCH_JACCARD)
    assert [[gdist.java_double(x) for x in r] for r in SJ] == case["sketch_D_jaccard"]


# ---------------------------------------------------------------- packing
PACK_MODES = {"default": {}, "set_major": {"pack_summary": 0},
              # chunks of ~1,000 windows: many chunk summaries, the upload of
              # chunk c + 1 overlapped with chunk c (or not)
              "chunked": {"pack_chunk": 1000}, "chunked_set_major": {"pack_chunk": 1000, "pack_summary": 0},
              "chunked_no_overlap": {"pack_chunk": 1000, "pack_overlap": 0},
              "chunked_pinned": {"pack_chunk": 1000, "pack_overlap": 2},
              # the code-major sort over code|set even where no window was skipped
              "chunked_full_key_sort": {"pack_chunk": 1000, "pack_code_sort": 0},
              # the codes buffer sized from the first chunk and grown (budget 0:
              # never the one buffer for every window)
              "grown": {"pack_chunk": 1000, "pack_codes_budget": 0},
              "grown_set_major": {"pack_chunk": 1000, "pack_codes_budget": 0, "pack_summary": 0}}


@pytest.mark.parametrize("mode", sorted(PACK_MODES))
@pytest.mark.parametrize("seed", range(6))
def test_pack_random_modes(ctx, opts, seed, mode):
    """Codes and offsets against the oracle: the code-major pack sort that
    keeps each chunk's dictionary summary (option pack_summary 1, the
    default), the set-major one (0), and both over many small chunks whose
    bytes upload while the previous chunk packs."""
    import gdist
    opts(**PACK_MODES[mode])
    rng = random.Random(seed)
    for _ in range(12):
        kind = rng.choice([0, 1])
        if kind == 0:
            alpha = rng.choice(["ACGT", "acgtACGT", "ACGTN", "ACGTNRYacgt", "ACGT\0"])
            flags = rng.choice([0, 1, 2]) | rng.choice([0, 4, 8])
            k = rng.randint(1, 21 if flags & 8 else 32)
        else:
            alpha = rng.choice(["ACDEFGHIKLMNPQRSTVWY", "ACDEFGHIKLMNPQRSTVWYX*", "acdefgACD", "ACD\0"])
            flags = rng.choice([0, 4, 8]) | rng.choice([0, 0x10])
            k = rng.randint(1, 12)
        seqs = ["".join(rng.choice(alpha) for _ in range(rng.randint(0, 300))) for _ in range(rng.randint(1, 40))]
        kt = gdist.KmerType.DNA if kind == 0 else gdist.KmerType.PROT
        try:
            eo, ec = oracle_pack(seqs, k, kind, flags)
        except ValueError:
            with pytest.raises(ValueError):
                gdist.KmerSets.from_sequences(seqs, k, kt, flags, ctx)
            continue
        sets = gdist.KmerSets.from_sequences(seqs, k, kt, flags, ctx)
        off, codes = sets.download()
        assert np.array_equal(off, eo) and np.array_equal(codes, ec), (kind, k, flags)


def test_pack_repetitive_small_k_grown(ctx, opts):
    """repetitive input with a small k (protein k=3 over a few
    residues: every set holds a few hundred distinct kmers of thousands of
    windows) packed in small chunks into the grown codes buffer: codes,
    offsets and the matrix equal the oracle."""
    import gdist
    rng = np.random.default_rng(5)
    seqs = [bytes(rng.choice(np.frombuffer(b"ACDEFG", np.uint8), 4000)) for _ in range(60)]
    opts(pack_chunk=20000, pack_codes_budget=0)
    sets = gdist.KmerSets.from_sequences(seqs, 3, gdist.KmerType.PROT, 0, ctx)
    eo, ec = oracle_pack(seqs, 3, 1, 0)
    off, codes = sets.download()
    assert np.array_equal(off, eo) and np.array_equal(codes, ec)
    assert len(ec) < 60 * 4000 / 10                  # far fewer unique codes than windows
    eI, eD = oracle.matrix(eo, ec, 0, 60, 0, 60)
    I, D = sets.matrix(method=gdist.METHOD_SORTED)
    assert np.array_equal(I, eI) and bits_equal(D, eD)


@pytest.mark.parametrize("mode", ["chunked", "chunked_set_major", "chunked_no_overlap", "chunked_pinned", "grown"])
def test_chunked_pack_bitset_matrix(ctx, opts, mode):
    """A collection packed in ~20 chunks (chunk summaries merged for the
    dictionary, uploads overlapped): codes, then the bitset matrix, equal the
    oracle's."""
    import gdist
    opts(**PACK_MODES[mode])
    opts(pack_chunk=40000)
    seqs = synth_sets(120, 4000, 0.01, 77)
    eo, ec = oracle_pack(seqs, 21, 0, 0)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    off, codes = sets.download()
    assert np.array_equal(off, eo) and np.array_equal(codes, ec)
    sets.build_bitsets()
    I, D = sets.matrix(method=gdist.METHOD_BITSET)
    eI, eD = oracle.matrix(eo, ec, 0, 120, 0, 120)
    assert np.array_equal(I, eI) and bits_equal(D, eD)


def test_pack_pinned_source_large(ctx):
    """Sequence bytes in a page-locked host buffer from gdist_host_alloc
    (gdist.HostBuffer) upload with one DMA per chunk: ~140 MB in two chunks,
    the first ending mid-sequence, pack the same codes as the same bytes in
    pageable memory (the runtime's staged copies) and as upload-first."""
    import gdist
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    lens = [1_000_000 + 37 * i for i in range(140)]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    flat = rng.choice(acgt, int(off[-1]))
    got = {}
    with gdist.HostBuffer(int(off[-1])) as hb:
        hb.array[:] = flat
        for name, blob, ov in (("pinned", hb.array, 1), ("pageable", flat, 1), ("first", flat, 0)):
            with ctx.options(pack_overlap=ov, pack_chunk=1 << 27):
                sets = gdist.KmerSets.from_blob(blob, off, 21, gdist.KmerType.DNA, 0, ctx)
            got[name] = sets.download()
            sets.free()
    for name in ("pageable", "first"):
        assert np.array_equal(got["pinned"][0], got[name][0]) and np.array_equal(got["pinned"][1], got[name][1])


def test_pack_rejects_unencodable_and_bad_k(ctx):
    import gdist
    with pytest.raises(ValueError):
        gdist.KmerSets.from_sequences(["ACGTX"], 5, gdist.KmerType.DNA, gdist.AMBIG_KEEP, ctx)
    with pytest.raises(ValueError):
        gdist.KmerSets.from_sequences(["ACGT"], 33, gdist.KmerType.DNA, 0, ctx)
    with pytest.raises(ValueError):
        gdist.KmerSets.from_sequences(["ACDE"], 13, gdist.KmerType.PROT, 0, ctx)
    with pytest.raises(ValueError):
        gdist.KmerSets.from_sequences(["AC1DE"], 10, gdist.KmerType.PROT, 0, ctx)


def test_empty_and_short_inputs(ctx):
    import gdist
    sets = gdist.KmerSets.from_sequences(["", "AC", "ACGTACGT", ""], 5, gdist.KmerType.DNA, 0, ctx)
    assert sets.sizes().tolist()[:2] == [0, 0]
    I, D = sets.matrix()
    assert I[0, 1] == 0 and D[0, 1] == 1.0 and D[0, 0] == 1.0
    _, Dn = sets.matrix(flags=gdist.EMPTY_NAN)
    assert math.isnan(Dn[0, 1]) and Dn[2, 2] == 0.0
    none = gdist.KmerSets.from_sequences([], 5, gdist.KmerType.DNA, 0, ctx)
    assert len(none) == 0
    I0, D0 = none.matrix()
    assert I0.shape == (0, 0)


# ---------------------------------------------------------------- matrices
def synth_sets(n, length, pmax, cfg, protein=False):
    from gdist import synth
    g = synth.genomes(n, length, pmax, cfg, protein=protein)
    return [bytes(r) for r in g]


@pytest.mark.parametrize("method", ["sorted", "bitset", "bitset_keep"])
def test_matrix_vs_oracle_rectangles(ctx, method):
    import gdist
    seqs = synth_sets(300, 3000, 0.05, 91)
    sets = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
    m = gdist.METHOD_SORTED
    if method != "sorted":
        sets.build_bitsets(keep_singletons=(method == "bitset_keep"))
        m = gdist.METHOD_BITSET
    off, codes = oracle_pack(seqs, 15, 0, 0)
    for (r0, r1, c0, c1, upper) in [(0, 300, 0, 300, True), (0, 300, 0, 300, False), (37, 201, 5, 290, False),
                                    (100, 101, 0, 300, False), (129, 260, 0, 300, True), (0, 1, 0, 1, False)]:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=upper, method=m)
        eI, eD = oracle.matrix(off, codes, r0, r1, c0, c1, flags=0x100 if upper else 0)
        if upper:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            assert (I[~mask] == -1).all() and np.isnan(D[~mask]).all()   # untouched
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI)
        assert bits_equal(D, eD)


def test_bitset_prune_equals_keep_and_dictionary(ctx):
    import gdist
    seqs = synth_sets(150, 5000, 0.01, 92)
    a = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    b = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    da, wa = a.build_bitsets(keep_singletons=False)
    db, wb = b.build_bitsets(keep_singletons=True)
    assert da < db
    Ia, Da = a.matrix(method=gdist.METHOD_BITSET)
    Ib, Db = b.matrix(method=gdist.METHOD_BITSET)
    Is, Ds = a.matrix(method=gdist.METHOD_SORTED)
    assert np.array_equal(Ia, Ib) and np.array_equal(Ia, Is)
    assert bits_equal(Da, Db) and bits_equal(Da, Ds)
    # dictionary with singletons == number of distinct kmers overall
    off, codes = oracle_pack(seqs, 21, 0, 0)
    assert db == len(np.unique(codes))


def test_protein_sorted_vs_oracle(ctx):
    import gdist
    seqs = synth_sets(200, 2000, 0.10, 93, protein=True)
    sets = gdist.KmerSets.from_sequences(seqs, 8, gdist.KmerType.PROT, 0, ctx)
    off, codes = oracle_pack(seqs, 8, 1, 0)
    I, D = sets.matrix(upper=True, method=gdist.METHOD_SORTED)
    eI, eD = oracle.matrix(off, codes, 0, 200, 0, 200, flags=0x100)
    iu = np.triu_indices(200, 1)
    assert np.array_equal(I[iu], eI[iu]) and bits_equal(D[iu], eD[iu])


def test_large_segments_and_sentinel_code(ctx):
    """Segments larger than one LDS table fill, and the all-ones code."""
    import gdist
    rng = np.random.default_rng(4)
    sets_codes = []
    base = np.unique(rng.integers(0, 2 ** 63, 30000, dtype=np.uint64))
    for t in range(5):
        keep = base[rng.random(len(base)) < 0.8]
        extra = np.array([~np.uint64(0)], dtype=np.uint64) if t % 2 == 0 else np.zeros(0, np.uint64)
        sets_codes.append(np.unique(np.concatenate([keep, extra])))
    off = np.zeros(6, np.int64)
    off[1:] = np.cumsum([len(c) for c in sets_codes])
    flat = np.concatenate(sets_codes)
    sets = gdist.KmerSets.from_codes(off, flat, 8, gdist.KmerType.PROT, ctx)
    I, D = sets.matrix(method=gdist.METHOD_SORTED)
    eI, eD = oracle.matrix(off, flat, 0, 5, 0, 5)
    assert np.array_equal(I, eI) and bits_equal(D, eD)
    sets.build_bitsets()
    I2, D2 = sets.matrix(method=gdist.METHOD_BITSET)
    assert np.array_equal(I2, eI) and bits_equal(D2, eD)


@pytest.mark.parametrize("fill", [0, 1, 2, 5])
@pytest.mark.parametrize("keep", [False, True])
def test_bitset_fill_ragged_sets(ctx, opts, fill, keep):
    """The bitset fills (merged positions + LDS row slices: one workgroup or
    one wave a segment; the sort; the one-pass atomics) on ragged sets: empty sets, two-code sets that span
    the whole dictionary (the merge gallops), sets far larger than a fill
    segment at unaligned offsets, and the all-ones code."""
    import gdist
    opts(fill_sort=fill)
    rng = np.random.default_rng(17 + fill)
    base = np.unique(rng.integers(0, 2 ** 63, 40000, dtype=np.uint64))
    sets_codes = []
    for t in range(23):
        if t % 7 == 3:
            c = np.zeros(0, np.uint64)
        elif t % 7 == 5:
            c = np.array([base[1], base[-2]], np.uint64)
        else:
            c = base[rng.random(len(base)) < rng.uniform(0.05, 0.95)]
            c = c[: len(c) - int(rng.integers(0, 5))]
        if t % 4 == 0:
            c = np.concatenate([c, np.array([~np.uint64(0)], np.uint64)])
        sets_codes.append(np.unique(c))
    off = np.zeros(len(sets_codes) + 1, np.int64)
    off[1:] = np.cumsum([len(c) for c in sets_codes])
    flat = np.concatenate(sets_codes)
    sets = gdist.KmerSets.from_codes(off, flat, 8, gdist.KmerType.PROT, ctx)
    sets.build_bitsets(keep_singletons=keep)
    n = len(sets_codes)
    I, D = sets.matrix(method=gdist.METHOD_BITSET)
    eI, eD = oracle.matrix(off, flat, 0, n, 0, n)
    assert np.array_equal(I, eI) and bits_equal(D, eD)


# ---------------------------------------------------------------- properties at size
def test_full_size_properties_bitset(ctx):
    """Size-independent properties on a larger collection: symmetry,
    diagonal I = |A|, D = 0 on the diagonal, and agreement with the oracle
    on a sampled row block."""
    import gdist
    n = 600
    seqs = synth_sets(n, 20000, 0.002, 94)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    I, D = sets.matrix(method=gdist.METHOD_BITSET)
    assert np.array_equal(I, I.T) and bits_equal(D, D.T)
    assert np.array_equal(np.diag(I), sets.sizes())
    assert (np.diag(D) == 0.0).all()
    off, codes = oracle_pack(seqs[:40], 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, 40, 0, 40)
    assert np.array_equal(I[:40, :40], eI) and bits_equal(D[:40, :40], eD)
    Is, Ds = sets.matrix((0, 64), (0, n), method=gdist.METHOD_SORTED)
    assert np.array_equal(Is, I[:64]) and bits_equal(Ds, D[:64])


def test_device_outputs_and_leading_dimension(ctx):
    import gdist
    seqs = synth_sets(130, 4000, 0.05, 95)
    sets = gdist.KmerSets.from_sequences(seqs, 12, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    ld = 200
    dI = ctx.alloc(130 * ld * 4)
    dD = ctx.alloc(130 * ld * 8)
    sets.matrix_device(dI.ptr, dD.ptr, ld, (0, 130), (0, 130), method=gdist.METHOD_BITSET)
    I = dI.to_host(np.int32).reshape(130, ld)[:, :130]
    D = dD.to_host(np.float64).reshape(130, ld)[:, :130]
    k_ms, call_ms, launches = ctx.last_timing()
    off, codes = oracle_pack(seqs, 12, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, 130, 0, 130)
    assert np.array_equal(I, eI) and bits_equal(D, eD)
    assert launches == 1 and 0 < k_ms <= call_ms


@pytest.mark.parametrize("method", ["sorted", "bitset", "sketch"])
def test_device_upper_leaves_lower_untouched(ctx, method):
    """GDIST_UPPER_TRIANGLE with device outputs: entries with j <= i keep the
    caller's values (gdist.h), on a row block that straddles the diagonal."""
    import gdist
    n, ld = 150, 160
    seqs = synth_sets(n, 4000, 0.02, 105)
    sets = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
    r0, r1, c0, c1 = 40, 110, 10, 150
    nr = r1 - r0
    dI, dD = ctx.alloc(nr * ld * 4), ctx.alloc(nr * ld * 8)
    dI.from_host(np.full(nr * ld, -7, np.int32))
    dD.from_host(np.full(nr * ld, 42.5))
    off, codes = oracle_pack(seqs, 15, 0, 0)
    if method == "sketch":
        sk = sets.sketches(64)
        sk.matrix_device(dI.ptr, dD.ptr, ld, (r0, r1), (c0, c1), upper=True)
        ref = [oracle.sketch(codes[off[i]:off[i + 1]], 15, 0, 64) for i in range(n)]
        eI = np.zeros((nr, c1 - c0), np.int32)
        eD = np.zeros((nr, c1 - c0))
        for a in range(nr):
            for b in range(c1 - c0):
                eD[a, b], eI[a, b] = oracle.sketch_distance(ref[r0 + a], ref[c0 + b], 64, 0)
    else:
        m = gdist.METHOD_SORTED if method == "sorted" else gdist.METHOD_BITSET
        if method == "bitset":
            sets.build_bitsets()
        sets.matrix_device(dI.ptr, dD.ptr, ld, (r0, r1), (c0, c1), upper=True, method=m)
        eI, eD = oracle.matrix(off, codes, r0, r1, c0, c1)
    I = dI.to_host(np.int32).reshape(nr, ld)[:, :c1 - c0]
    D = dD.to_host(np.float64).reshape(nr, ld)[:, :c1 - c0]
    up = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (nr, c1 - c0))
    assert np.all(I[~up] == -7) and np.all(D[~up] == 42.5)
    assert np.array_equal(I[up], eI[up]) and bits_equal(D[up], eD[up])
    pad = dI.to_host(np.int32).reshape(nr, ld)[:, c1 - c0:]
    assert np.all(pad == -7)


# ---------------------------------------------------------------- row queries
def test_row_queries(ctx):
    import gdist
    seqs = synth_sets(80, 3000, 0.2, 96)
    sets = gdist.KmerSets.from_sequences(seqs, 11, gdist.KmerType.DNA, 0, ctx)
    off, codes = oracle_pack(seqs, 11, 0, 0)
    _, D = oracle.matrix(off, codes, 0, 80, 0, 80)          # expectations from the CPU oracle
    cols = [5, 17, 3, 60, 22, 79]
    for use_bits in (False, True):
        if use_bits:
            sets.build_bitsets()
        d = sets.row_query(9, cols)
        assert bits_equal(d, D[9, cols])
        t = float(np.median(D[9, cols]))
        assert sets.row_query(9, cols, gdist.QUERY_ANY_LE, t) == bool((D[9, cols] <= t).any())
        assert sets.row_query(9, cols, gdist.QUERY_ANY_LE, -1.0) is False
        pos, bd = sets.row_query(9, cols, gdist.QUERY_ARGMIN)
        assert pos == int(np.argmin(D[9, cols])) and bd == D[9, cols].min()
    far = gdist.KmerSets.from_sequences(["AAAAAAAAAAAAAAAA", "CCCCCCCCCCCCCCCC"], 11, gdist.KmerType.DNA, 0, ctx)
    assert far.row_query(0, [1], gdist.QUERY_ARGMIN) == (-1, 1.0)      # NULL_RESULT semantics


@pytest.mark.parametrize("T", [0, 8, 1000])
def test_row_query_repeated_columns(ctx, T):
    """A column set listed twice gets the same distance at both positions, on
    the dense and the rare tier (a set's rare counts are gathered per
    position, not scattered per set)."""
    import gdist
    n = 120
    seqs = synth_sets(n, 5000, 0.01, 104)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    off, codes = oracle_pack(seqs, 21, 0, 0)
    _, eD = oracle.matrix(off, codes, 0, n, 0, n)
    sets.build_bitsets(rare_threshold=T)
    cols = [7, 30, 7, 119, 30, 30, 0, 55]
    for q in (7, 55, 90):
        d = sets.row_query(q, cols)
        assert bits_equal(d, eD[q, cols]), (T, q)


def test_sequence_kmers_view_api(ctx):
    import gdist
    a = gdist.KmerType.DNA.createKmers("ACGTTGCAACGTAGCTAGCT", 5)
    b = gdist.KmerType.DNA.createKmers("ACGTTGCAACGTAGCTTTTT", 5)
    sa = pyref.kmer_set("ACGTTGCAACGTAGCTAGCT", 5)
    sb = pyref.kmer_set("ACGTTGCAACGTAGCTTTTT", 5)
    assert a.size() == len(sa) and b.size() == len(sb)
    assert a.distance(b) == pyref.set_distance(sa, sb)
    assert a.similarity(b) == len(sa & sb)
    assert a.hashSet(8).tolist() == pyref.sketch(sa, 8)


# ---------------------------------------------------------------- sketches
def test_sketch_matrix_vs_oracle(ctx):
    import gdist
    seqs = synth_sets(70, 2000, 0.1, 97)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    off, codes = oracle_pack(seqs, 21, 0, 0)
    for w in (50, 1000, 1500):
        sk = sets.sketches(w)
        so, sv = sk.download()
        ref = [oracle.sketch(codes[off[i]:off[i + 1]], 21, 0, w) for i in range(70)]
        for i in range(70):
            assert np.array_equal(sv[so[i]:so[i + 1]], ref[i])
        for fl in (0, gdist.SKETCH_JACCARD):
            C, D = sk.matrix(upper=True, flags=fl)
            for i in range(0, 70, 7):
                for j in range(i + 1, 70):
                    d, c = oracle.sketch_distance(ref[i], ref[j], w, fl)
                    assert C[i, j] == c and D[i, j] == d
    up = gdist.SketchSets.from_signatures([np.array([1, 5, 9], np.int32), np.array([5, 9, 11], np.int32)], 4, ctx)
    C, D = up.matrix()
    assert C[0, 1] == 2 and D[0, 1] == pyref.sketch_distance([1, 5, 9], [5, 9, 11], 4)[0]


@pytest.mark.parametrize("phase,cap,ring,v2,k", [
    (1, None, None, 1, 2), (1, 2, 512, 1, 2), (1, 7, 512, 1, 2), (1, 64, 256, 1, 2), (1, 255, 256, 1, 2),
    (1, 5000, 128, 1, 2), (1, 15, 16, 1, 2), (1, 8, 32, 1, 2), (1, 120, 512, 1, 2), ("w", 15, 16, 1, 2),
    ("w", 8, 32, 1, 2), ("w", 64, 256, 1, 2), ("p0", None, None, 1, 2), ("p0", 64, 256, 1, 2),
    (0, 300, None, 1, 2), (0, 300, None, 0, 2), (0, 300, None, 0, 4), (0, 300, None, 0, 1)])
def test_sketch_merge_edges_vs_oracle(ctx, opts, phase, cap, ring, v2, k):
    """Uploaded sketches with the merge's edge cases, every pair against the
    oracle, every merge loop (the ring kernel, the default: options
    sketch_ring + sketch_cap, rings of 16..512 slots with 2..5000 steps per
    phase; pairs without room in a small ring take global-memory steps, or
    with sketch_wait wait for the slower pairs until a phase makes no
    progress; sketch_phase = 0 with sketch_v2 / sketch_k: whole sketches in
    LDS; p0: 256-slot rings addressed by AND + shift-add instead of one
    v_perm_b32, option sketch_perm 0): empty and short sketches,
    identical ones, disjoint ones, INT_MIN / INT_MAX hashes (INT_MAX is the
    LDS sentinel: such pairs take the checked loop)."""
    import gdist
    wait = phase == "w"                       # ring pairs without room wait (option sketch_wait)
    perm0 = phase == "p0"
    opts(sketch_phase=1 if (wait or perm0) else phase, sketch_wait=1 if wait else None, sketch_cap=cap,
         sketch_ring=ring, sketch_v2=v2, sketch_k=k, sketch_perm=0 if perm0 else None)
    rng = np.random.default_rng(1234)
    for w in (64, 1000):
        sk = []
        for t in range(96):
            n = [0, 1, 2, w // 2, w - 1, w, w, w][t % 8]
            lo, hi = (-2**31, 2**31 - 1) if t % 3 else (-2**31, -2**31 + 40 * w)
            v = np.unique(rng.integers(lo, hi, size=3 * n + 8, endpoint=True, dtype=np.int64))
            v = np.sort(rng.choice(v, size=min(n, len(v)), replace=False)).astype(np.int32)
            if t % 11 == 0 and n:
                v[-1] = 2**31 - 1
                v = np.unique(v)
            if t % 13 == 0 and n:
                v[0] = -2**31
                v = np.unique(v)
            sk.append(v)
        sk[10] = sk[9].copy()                                     # identical pair
        sk[20] = np.arange(w, dtype=np.int32) * 2                 # disjoint interleaved pair
        sk[21] = np.arange(w, dtype=np.int32) * 2 + 1
        S = gdist.SketchSets.from_signatures(sk, w, ctx)
        for fl in (0, gdist.SKETCH_JACCARD):
            C, D = S.matrix(flags=fl)
            for i in range(len(sk)):
                for j in range(len(sk)):
                    d, c = oracle.sketch_distance(sk[i], sk[j], w, fl)
                    assert C[i, j] == c and bits_equal(np.array([D[i, j]]), np.array([d])), (w, fl, i, j)


# ---------------------------------------------------------------- processors
def test_fasta_distance_processor_output(ctx):
    import gdist
    from gdist import processors
    seqs = synth_sets(40, 800, 0.05, 98)
    recs = [gdist.Sequence(f"s{i}", f"genome {i}", s.decode()) for i, s in enumerate(seqs)]
    buf = io.StringIO()
    pairs = processors.fasta_distance(recs, buf, kmer_size=13, ctx=ctx)
    assert pairs == 40 * 39 // 2
    lines = buf.getvalue().splitlines()
    assert lines[0] == "seq1\tname1\tseq2\tname2\tdistance"
    sets = [pyref.kmer_set(s.decode(), 13) for s in seqs]
    exp = {f"s{i}\tgenome {i}\ts{j}\tgenome {j}\t{pyref.java_double_str(pyref.set_distance(sets[i], sets[j]))}"
           for i in range(40) for j in range(i + 1, 40)}
    assert set(lines[1:]) == exp
    with pytest.raises(processors.ParseFailureException):
        processors.fasta_distance(recs, io.StringIO(), kmer_size=1, ctx=ctx)


def test_genome_and_reps_processors(ctx):
    from gdist import processors
    seqs = synth_sets(30, 1500, 0.3, 99)
    gens = [processors.Genome(f"g{i}", f"name {i}", [s[:700].decode(), s[700:].decode()]) for i, s in enumerate(seqs)]
    buf = io.StringIO()
    n = processors.genome_distance(gens[:10], [gens[10:20], gens[20:]], buf, kmer_size=12, ctx=ctx)
    assert n == 20 * 10
    lines = buf.getvalue().splitlines()
    ks = [pyref.kmer_set("\0".join(g.contigs), 12) for g in gens]
    # every line, in the reference's order: comparison genomes in directory
    # order, each against every base genome (GenomeProcessor.java:119-146)
    exp = [f"g{j}\tg{i}\t{pyref.java_double_str(pyref.set_distance(ks[j], ks[i]))}"
           for j in range(10, 30) for i in range(10)]
    assert lines[1:] == exp
    prefix, lst, stats = processors.distance_reps(gens, kmer_size=12, max_dist=0.5, ctx=ctx)
    assert prefix == "rep0.5000_K12"
    reps = []
    for i in range(30):                        # greedy pass-1 restated on string sets
        if not any(pyref.set_distance(ks[r], ks[i]) <= 0.5 for r in reps):
            reps.append(i)
    rows = [l.split("\t") for l in lst.splitlines()[1:]]
    assert len(rows) == 30
    rep_ids = {f"g{r}" for r in reps}
    for i, row in enumerate(rows):
        d = min(pyref.set_distance(ks[i], ks[r]) for r in reps)
        assert row[2] in rep_ids and row[4] == pyref.java_double_str(0.0 if i in reps else d)


@pytest.mark.parametrize("block", [None, "100", "37"])
def test_greedy_reps_device(ctx, block, opts):
    """gdist_greedy_reps: pass 1 equals the sequential loop of row queries
    (DistanceRepsProcessor.java:185-200) for one block and several; pass 2
    equals the argmin over representatives of the exact distances, ties to
    the lowest tie rank, on a collection with duplicated genomes (exact ties)."""
    import gdist
    if block:
        opts(reps_block=int(block))
    base = synth_sets(150, 3000, 0.15, 109)
    seqs = base + [base[i] for i in (3, 17, 40, 41, 99)]           # duplicates -> ties
    n = len(seqs)
    sets = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
    off, codes = oracle_pack(seqs, 15, 0, 0)
    _, D = oracle.matrix(off, codes, 0, n, 0, n)             # expectations from the CPU oracle
    for t in (0.3, 0.6):
        reps = []
        for k in range(n):
            if not any(D[k, r] <= t for r in reps):
                reps.append(k)
        for method in (gdist.METHOD_SORTED, gdist.METHOD_BITSET):
            is_rep = sets.greedy_reps(t, method=method)
            assert [int(i) for i in np.flatnonzero(is_rep)] == reps, (t, method)
        rank = np.random.default_rng(5).permutation(n).astype(np.int64)
        is_rep, rep_of, rep_d = sets.greedy_reps(t, assign=True, tie_rank=rank)
        for k in range(n):
            if k in reps:
                assert rep_of[k] == k and rep_d[k] == 0.0
                continue
            cand = [r for r in reps if D[k, r] < 1.0]
            best = min(cand, key=lambda r: (D[k, r], rank[r]))
            assert rep_of[k] == best and bits_equal(rep_d[k], D[k, best]), (t, k)


def test_reps_processors_java_semantics(ctx):
    """distReps breaks pass-2 ties in repMap's HashMap order; fastaReps with a
    repeated label replaces the representative under that key (HashMap.put)."""
    import gdist
    from gdist import processors as P
    base = synth_sets(12, 2000, 0.4, 110)
    seqs = base + [base[2], base[2], base[5]]
    ids = [f"fig|{1000 + 37 * i}.peg.{i}" for i in range(len(seqs))]
    gens = [P.Genome(ids[i], f"n{i}", [s.decode()]) for i, s in enumerate(seqs)]
    _, lst, _ = P.distance_reps(gens, kmer_size=12, max_dist=0.6, ctx=ctx)
    ks = [pyref.kmer_set(s.decode(), 12) for s in seqs]
    reps = []
    for i in range(len(seqs)):
        if not any(pyref.set_distance(ks[r], ks[i]) <= 0.6 for r in reps):
            reps.append(i)
    order = [reps[o] for o in P.java_hashmap_order([ids[r] for r in reps], P.DISTREPS_REPMAP_CAPACITY)]
    rows = [l.split("\t") for l in lst.splitlines()[1:]]
    for i, row in enumerate(rows):
        if i in reps:
            assert row[2] == ids[i] and row[4] == "0.0"
            continue
        best, bd = None, 1.0                    # reduce(NULL_RESULT, merge): left wins ties
        for r in order:
            d = pyref.set_distance(ks[i], ks[r])
            if not (bd <= d):
                best, bd = r, d
        assert row[2] == ids[best] and row[4] == pyref.java_double_str(bd), i
    # fastaReps, repeated label
    recs = [gdist.Sequence("a", "x0", "ACGTACGTTTGACCAGT" * 8), gdist.Sequence("b", "x1", "TTTTGGGGCCCCAAAA" * 8),
            gdist.Sequence("a", "x2", "GATTACAGATTACAGG" * 8), gdist.Sequence("c", "x3", "ACGTACGTTTGACCAGT" * 8)]
    out = io.StringIO()
    reps = P.fasta_reps(recs, out, kmer_size=8, max_dist=0.5, ctx=ctx)
    # "a" (x0) is replaced by x2 under key "a", so x3 (equal to x0) finds no representative
    assert out.getvalue().splitlines() == ["seq\tname", "a\tx0", "b\tx1", "a\tx2", "c\tx3"]
    assert reps == [2, 1, 3]


def test_bitset_row_blocks_like_ranks(ctx):
    """Row blocks as the multi-GPU partition hands them out (r0 > 0, all
    columns, upper; aligned to the 128-set tiles or not) and upper
    rectangles with c0 > 0: the column tile grid starts at an origin
    = r0 (mod 128) so diagonal tiles run the trimmed variant; every pair exact."""
    import gdist
    n = 700
    seqs = synth_sets(n, 3000, 0.01, 112)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    off, codes = oracle_pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n)
    sets.build_bitsets()
    for (r0, r1, c0, c1) in [(0, 256, 0, n), (256, 512, 0, n), (512, 700, 0, n), (300, 450, 0, n),
                             (77, 301, 0, n), (100, 300, 50, 700), (400, 650, 133, 690), (5, 60, 0, 40)]:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=True, method=gdist.METHOD_BITSET)
        up = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
        assert np.array_equal(I[up], eI[r0:r1, c0:c1][up]), (r0, r1, c0, c1)
        assert bits_equal(D[up], eD[r0:r1, c0:c1][up]), (r0, r1, c0, c1)


def test_bitset_partial_row_tiles(ctx, opts):
    """A block whose last row tile holds 1..127 rows runs it through the
    launches instantiated for RR = ceil(rows / 16) accumulator rows: every RR
    (1..7, RR = 7 enabled here) and its boundaries, upper (diagonal +
    off-diagonal partial tiles) and full rectangles, exact against the oracle."""
    import gdist
    opts(bitset_partial_rr=7)
    n = 420
    seqs = synth_sets(n, 2500, 0.01, 113)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    off, codes = oracle_pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n)
    sets.build_bitsets()
    for m in (1, 15, 16, 17, 33, 48, 63, 64, 65, 80, 97, 111, 112, 113, 127):
        for (r0, up) in ((0, True), (3, True), (150, True), (131, False)):
            r1 = min(n, r0 + 128 + m)
            c0, c1 = (0, n) if up else (40, 400)
            I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
            mask = (np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0)) if up
                    else np.ones((r1 - r0, c1 - c0), bool))
            assert np.array_equal(I[mask], eI[r0:r1, c0:c1][mask]), (m, r0, up)
            assert bits_equal(D[mask], eD[r0:r1, c0:c1][mask]), (m, r0, up)


@pytest.mark.parametrize("strand", [0, 0x1, 0x2])
def test_k32_all_ones_code(ctx, strand):
    """DNA k=32 uses all 64 code bits: the poly-T kmer is ~0, the sorted
    join's empty-slot sentinel (handled by its has-empty-key flag). Every
    path must count it like any other kmer."""
    import gdist
    rng = np.random.default_rng(111)
    polyT = "T" * 40
    seqs = []
    for i in range(24):
        body = "".join(rng.choice(list("ACGT"), 300))
        seqs.append((body[:150] + (polyT if i % 3 else "") + body[150:] + ("A" * 33 if i % 4 == 0 else "")).encode())
    off, codes = oracle_pack(seqs, 32, 0, strand)
    # canonical mode keeps min(poly-T, poly-A) = poly-A: ~0 cannot occur there
    assert (np.asarray(codes) == np.uint64(2**64 - 1)).any() == (strand != 0x2)
    eI, eD = oracle.matrix(off, codes, 0, 24, 0, 24)
    sets = gdist.KmerSets.from_sequences(seqs, 32, gdist.KmerType.DNA, strand, ctx)
    for m in (gdist.METHOD_SORTED, gdist.METHOD_BITSET):
        I, D = sets.matrix(method=m)
        assert np.array_equal(I, eI) and bits_equal(D, eD), m
    for keep in (False, True):
        # every fill route: the hash fill's empty marker is the code ~0 itself
        # (kept out of band), the windows, the sort
        for fill in (None, 4, 0, 5, 1):
            with ctx.options(fill_sort=fill):
                sets.build_bitsets(keep_singletons=keep)
            I, D = sets.matrix(method=gdist.METHOD_BITSET)
            assert np.array_equal(I, eI) and bits_equal(D, eD), (keep, fill)
    d = sets.row_query(1, list(range(24)))
    assert bits_equal(d, eD[1])


# ---------------------------------------------------------------- two-tier dictionary
@pytest.mark.parametrize("dedup", ["1", "0"])
@pytest.mark.parametrize("kernel", ["0", "1", "1w", "1l", "1lw", "1x", "1d", "1dw", "1n"])
@pytest.mark.parametrize("T", [0, 3, 8, 1000])
def test_rare_tier_thresholds_exact(ctx, T, kernel, dedup, opts):
    """Dense-only (T=0), mixed, and all-rare (T > N) dictionaries give the
    same bit-exact counts and distances as the oracle, through the list-major
    (0) and the row-major (1: 2-byte list members, 1w: 4-byte; 512-thread
    workgroups, 256 as 1l / 1lw, 1,024 as 1x; 1d / 1dw: every record once,
    members added to I by atomics, option rare_direct — C4's wide rows; the
    LDS walk's counters 16-bit by default, 1n: 32-bit, option rare_c16) rare kernel,
    with identical posting lists merged into weighted lists (1) or one list
    per kmer (0). T > N puts lists of up to N members in the rare tier: the
    wave-cooperative long-list walks."""
    import gdist
    opts(rare_kernel=int(kernel[0]), rare_dedup=int(dedup), rare_u16=0 if kernel.endswith("w") else None,
         rare_rows_threads=256 if "l" in kernel else 1024 if "x" in kernel else None,
         rare_direct=1 if "d" in kernel else None, rare_c16=0 if "n" in kernel else None)
    n = 200
    seqs = synth_sets(n, 6000, 0.01, 101)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets(rare_threshold=T)
    thr, lists, recs = sets.rare_info()
    assert thr == T
    kmers = sets.rare_kmers()
    if T > 2:
        assert lists > 0 and recs >= 2 * lists
        # shared substitutions give every covering kmer the same holders
        if dedup == "0":
            assert lists == kmers
        else:
            assert lists < (kmers / 4 if T < n else kmers)
    else:
        assert lists == 0
    incs, max_list = sets.rare_stats()
    assert max_list <= max(T - 1, 0) and (incs > 0) == (lists > 0)
    if T == 1000:
        assert max_list >= 64          # long lists take the wave path
    off, codes = oracle_pack(seqs, 21, 0, 0)
    for (r0, r1, c0, c1, up) in [(0, n, 0, n, False), (0, n, 0, n, True), (17, 150, 3, 190, False),
                                 (60, 61, 0, n, False)]:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
        eI, eD = oracle.matrix(off, codes, r0, r1, c0, c1, flags=0x100 if up else 0)
        if up:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI), (T, r0, r1, c0, c1, up)
        assert bits_equal(D, eD)
    cols = [5, 199, 0, 77, 150]
    d = sets.row_query(77, cols)
    _, eD = oracle.matrix(off, codes, 77, 78, 0, n)
    assert bits_equal(d, eD[0, cols])


@pytest.mark.parametrize("c16", [None, 0])
def test_rare_rows_heavy_rows_exact(ctx, opts, c16):
    """The row-major rare walk's 16-bit LDS counters (round 5, option
    rare_c16) are used only while every row's rare weight stays below 2^16:
    six 120 kbp genomes of one ancestor with rare_t 7 put every shared kmer
    (~240 K a genome, both strands) in the rare tier, merged into a few
    heavy lists, so a row weighs > 65,536 and the walk must keep 32-bit
    counters; counts and distances equal the oracle."""
    import gdist
    opts(rare_kernel=1, rare_c16=c16)
    n = 6
    seqs = synth_sets(n, 120_000, 0.002, 141)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets(rare_threshold=7)
    assert sets.rare_kmers() > 65536
    off, codes = oracle_pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n, flags=0, nthreads=4)
    assert eI[0, 1] > 65536                          # the premise: pair counts past 2^16
    for up in (True, False):
        I, D = sets.matrix(upper=up, method=gdist.METHOD_BITSET)
        iu = np.triu_indices(n, 1) if up else np.where(np.ones((n, n), bool))
        assert np.array_equal(I[iu], eI[iu]), (c16, up)
        assert bits_equal(D[iu], eD[iu])


SPARSE_MODES = {
    "auto": {},
    # the dense tiles issued before the sparse launch (option dense_first)
    "dense_first": {"sparse_zmax": 12, "sparse_fold": 0, "dense_first": 1},
    "all_sparse": {"sparse_zmax": 100000}, "mixed": {"sparse_zmax": 12},
    "no_locus": {"locus_order": 0, "sparse_zmax": 40}, "off": {"sparse": 0},
    # chunks flush with atomics (no partials within a zero budget)
    "atomic_flush": {"sparse_zmax": 100000, "sparse_part_budget": 0, "sparse_chunks": 5},
    # 1 x 2 micro-tiles (option sparse_mt 1) with 2 / 3 / 4 slots per lane in flight
    "rows_sun2": {"sparse_zmax": 40, "sparse_mt": 1, "sparse_sun": 2},
    "sun4": {"sparse_zmax": 100000, "sparse_mt": 1, "sparse_sun": 4, "sparse_chunks": 7},
    "sun3": {"sparse_zmax": 100000, "sparse_mt": 1, "sparse_sun": 3},
    "mt1_default": {"sparse_mt": 1},
    # a tile workgroup's waves take equal runs of words instead of claiming batches in turn
    "dyn_off": {"sparse_zmax": 100000, "sparse_dyn": 0},
    "dyn_off_default": {"sparse_dyn": 0, "sparse_chunks": 5},
    # 2 x 2 micro-tiles off the diagonal (default; row-trimmed tiles of the
    # unaligned regions below keep 1 x 2) with 4 / 3 (default) / 2 slots
    "mt2": {"sparse_zmax": 100000, "sparse_mt": 2, "sparse_sun": 4},
    "mt2_sun3": {"sparse_zmax": 100000, "sparse_mt": 2, "sparse_sun": 3, "sparse_chunks": 7},
    "mt2_sun2_atomic": {"sparse_zmax": 100000, "sparse_mt": 2, "sparse_sun": 2, "sparse_part_budget": 0,
                        "sparse_chunks": 3},
    # row-trimmed tiles (the unaligned regions below) in 1 x 2 micro-tiles (option sparse_rpart22 0)
    "rpart12": {"sparse_zmax": 100000, "sparse_rpart22": 0},
    # 2 x 2 off the diagonal, one product a slot on it (option sparse_diag22 0)
    "diag11": {"sparse_zmax": 100000, "sparse_diag22": 0},
    "diag11_default": {"sparse_diag22": 0},
    "sun2_atomic": {"sparse_zmax": 100000, "sparse_sun": 2, "sparse_part_budget": 0, "sparse_chunks": 3},
    # the dense words counted inside the tile kernel, 8 per chunk (partials / atomic flush),
    # or by their own tile launch
    "mixed_slabs": {"sparse_zmax": 12, "sparse_fold": 100000},
    "mixed_slabs_atomic": {"sparse_zmax": 12, "sparse_fold": 100000, "sparse_part_budget": 0},
    "mixed_tiles": {"sparse_zmax": 12, "sparse_fold": 0},
    # the default step is fused (tiles + a reduce that adds the rare pairs and
    # stores I and D); the same counts with zeroing + rare kernel + epilogue apart
    "unfused": {"sparse_fused": 0},
    "rare_kernel": {"sparse_rare": 0},
    "unfused_rare_kernel": {"sparse_fused": 0, "sparse_rare": 0},
    # the bitset fill by the (code, set) sort + run ranks, or by the one-pass
    # windowed searches with global atomics, instead of merged positions + LDS slices
    "fill_sort": {"fill_sort": 1},
    "fill_direct": {"fill_sort": 2},
    "fill_hash": {"fill_sort": 4},
    # the pack's two (code, set) pair sorts instead of one sort of set|code keys
    "pack_pairs": {"pack_sort": 1},
    # the pack without chunk summaries: the bitset build sorts every code for its dictionary
    "pack_nosummary": {"pack_summary": 0},
    # the pack's and the dictionary's radix sorts in 10-bit onesweep passes
    "sort_radix10": {"sort_radix": 10},
    "many_chunks": {"sparse_zmax": 100000, "sparse_chunks": 37},
    "mt2_sun2": {"sparse_zmax": 100000, "sparse_sun": 2, "sparse_chunks": 5},
    # chunk c of every tile on XCD c mod 8 (option sparse_xcd), with a chunk
    # count that leaves empty workgroups in the last group of 8, and atomics
    "xcd": {"sparse_zmax": 100000, "sparse_xcd": 1, "sparse_chunks": 13},
    "xcd_default": {"sparse_xcd": 1},
    "xcd_atomic": {"sparse_zmax": 100000, "sparse_xcd": 1, "sparse_part_budget": 0, "sparse_chunks": 6},
    # a dense-only dictionary: the substitution kmers two or more sets share
    # are dense too, and their words are counted from the set bits
    # (positive-sparse) beside the complement words
    "two_sided": {"rare_t": 2, "guides": 4},
}


_SPARSE_CASE = {}


def sparse_case():
    """The sweep's collection (300 x 20 kbp, p 0.003, seed 105) with the
    oracle's whole N x N matrix, computed once: the settings below share it
    (the oracle's matrices were most of each setting's time)."""
    if not _SPARSE_CASE:
        n = 300
        seqs = synth_sets(n, 20000, 0.003, 105)
        off, codes = oracle_pack(seqs, 21, 0, 0)
        eI, eD = oracle.matrix(off, codes, 0, n, 0, n, flags=0, nthreads=8)
        _SPARSE_CASE.update(n=n, seqs=seqs, eI=eI, eD=eD)
    return _SPARSE_CASE


@pytest.mark.parametrize("mode", list(SPARSE_MODES))
def test_sparse_complement_words_exact(ctx, mode, opts):
    """The dense tier in locus order with complement-sparse words: counts and
    distances are bit-exact against the oracle over upper triangles,
    rectangles, unaligned row blocks (as ranks get them) and row queries,
    whether every word is sparse, words are split between the sparse kernel
    and the tiles, the locus order is off (code order), or the split is off."""
    import gdist
    settings = SPARSE_MODES
    opts(**settings.get(mode, {}))
    case = sparse_case()
    n, seqs, fI, fD = case["n"], case["seqs"], case["eI"], case["eD"]
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    _, W = sets.build_bitsets()
    ws, wd, ent = sets.sparse_info()
    if mode in ("all_sparse", "atomic_flush", "many_chunks", "sun4", "sun3", "sun2_atomic", "mt2", "mt2_sun3",
                "mt2_sun2_atomic", "dyn_off", "diag11", "rpart12"):
        assert ws > 0 and wd == 0 and ent > 0
    elif mode in ("mixed", "mixed_slabs", "mixed_slabs_atomic", "mixed_tiles", "dense_first"):
        assert ws > 0 and wd > 0
    elif mode == "off":
        assert ws == 0 and wd == W
    elif mode == "two_sided":
        cw, pw = sets.sparse_sides()
        assert ws > 0 and cw > 0 and pw > 0 and cw + pw == ws
    for (r0, r1, c0, c1, up) in [(0, n, 0, n, True), (0, n, 0, n, False), (37, 211, 5, 290, False),
                                 (130, 259, 0, n, True), (299, 300, 0, n, False)]:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
        eI, eD = fI[r0:r1, c0:c1], fD[r0:r1, c0:c1]
        if up:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI), (mode, r0, r1, c0, c1, up)
        assert bits_equal(D, eD)
    cols = [4, 299, 0, 150, 150]
    d = sets.row_query(150, cols)
    assert bits_equal(d, fD[150, cols])


def test_sparse_equals_dense_at_size(ctx, opts):
    """C2-shaped collection (shared core, sparse substitutions): the whole
    triangle through the complement-sparse words equals the plain AND+popcount
    tiles pair for pair, and the oracle over the whole triangle; row-sharded blocks
    (unaligned, as ranks get them) agree too."""
    import gdist
    n = 420
    seqs = synth_sets(n, 200_000, 0.002, 106)
    sp = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sp.build_bitsets()
    ws, wd, ent = sp.sparse_info()
    assert ws > 0 and ent > 0
    I, D = sp.matrix(upper=True, method=gdist.METHOD_BITSET)
    opts(sparse=0)
    de = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    de.build_bitsets()
    assert de.sparse_info()[0] == 0
    eI, eD = de.matrix(upper=True, method=gdist.METHOD_BITSET)
    iu = np.triu_indices(n, 1)
    assert np.array_equal(I[iu], eI[iu]) and bits_equal(D[iu], eD[iu])
    opts(sparse=None)
    for (r0, r1) in [(0, 77), (77, 200), (200, 331), (331, 420)]:
        Ib, _ = sp.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
        mask = np.fromfunction(lambda a, b: b > (r0 + a), (r1 - r0, n))
        assert np.array_equal(Ib[mask], eI[r0:r1][mask]), (r0, r1)
    off, codes = oracle_pack(seqs, 21, 0, 0)
    oI, oD = oracle.matrix(off, codes, 0, n, 0, n, flags=0x100, nthreads=8)
    assert np.array_equal(I[iu], oI[iu]) and bits_equal(D[iu], oD[iu])


@pytest.mark.parametrize("mfma", [None, "nibble", "km2_group", "km2_ns3", "km2_ns4", "raw_group", "raw_km2",
                                  "raw_km2_ns3", "store", "sched0", "sched1_split3", "plane0", 0])
@pytest.mark.parametrize("T", [0, 3])
def test_dense_tiles_mfma_exact(ctx, opts, mfma, T):
    """The dense tier's tiles on the matrix cores (FP4 MFMA, 256 x 256 pairs
    a workgroup; default from 64 dense words) and by AND+popcount (option
    bitset_mfma 0): counts and distances bit-exact against the oracle over
    upper triangles, whole squares, rectangles, row blocks not aligned to a
    tile, partial tiles and one row; dense-only (T = 0) and with rare lists;
    the default stages of the bitsets themselves (nibbles made in registers,
    round 5) and the FP4 nibble operand (option bitset_mfma_raw 0) with
    4-word stages, 2-word stages with the tiles in 2 x 4 blocks, and rings
    of 3 and 4 stages (options bitset_mfma_km, bitset_mfma_group,
    bitset_mfma_ns); raw stages of 8 words (a 64 KiB ring, bitset_mfma_km 2)
    in rings of 2 and 3; one K split storing its counts, the rare tier after
    it (option bitset_mfma_store); the raw stages' DMA spread between the
    MFMAs with one barrier a stage (round 6, default; also over three K
    splits) and round 5's schedule (option bitset_mfma_sched 0); bit-plane
    operands under per-step e8m0 scales (round 6, default) and the nibbles
    of one dword a step (plane0: option bitset_mfma_plane 0)."""
    import gdist
    if mfma == "plane0":
        opts(bitset_mfma=1, bitset_mfma_plane=0, sparse=0)
    elif mfma and str(mfma).startswith("sched"):
        opts(bitset_mfma=1, bitset_mfma_sched=int(mfma[5]), sparse=0,
             bitset_mfma_splits=3 if mfma.endswith("split3") else None)
    elif mfma == "store":
        opts(bitset_mfma=1, bitset_mfma_store=1, sparse=0)
    elif mfma == "raw_km2":
        opts(bitset_mfma=1, bitset_mfma_km=2, sparse=0)
    elif mfma == "raw_km2_ns3":
        opts(bitset_mfma=1, bitset_mfma_km=2, bitset_mfma_ns=3, sparse=0)
    elif mfma == "nibble":
        opts(bitset_mfma=1, bitset_mfma_raw=0, sparse=0)
    elif mfma == "raw_group":
        opts(bitset_mfma=1, bitset_mfma_group=2, sparse=0)
    elif mfma == "km2_group":
        opts(bitset_mfma=1, bitset_mfma_raw=0, bitset_mfma_km=2, bitset_mfma_group=2, sparse=0)
    elif mfma in ("km2_ns3", "km2_ns4"):                # 3 / 4 stages in the ring
        opts(bitset_mfma=1, bitset_mfma_raw=0, bitset_mfma_km=2, bitset_mfma_ns=int(mfma[-1]), sparse=0)
    else:
        opts(bitset_mfma=mfma, sparse=0)
    n = 530
    seqs = synth_sets(n, 3000, 0.10, 111, protein=True)
    sets = gdist.KmerSets.from_sequences(seqs, 8, gdist.KmerType.PROT, 0, ctx)
    _, W = sets.build_bitsets(rare_threshold=T)
    assert W >= 64, W
    off, codes = oracle_pack(seqs, 8, 1, 0)
    for (r0, r1, c0, c1, up) in [(0, n, 0, n, True), (0, n, 0, n, False), (37, 300, 5, 510, False),
                                 (256, 530, 0, n, True), (100, 357, 100, 357, True), (529, 530, 0, n, False)]:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
        eI, eD = oracle.matrix(off, codes, r0, r1, c0, c1, flags=0x100 if up else 0)
        if up:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI), (mfma, T, r0, r1, c0, c1, up, np.flatnonzero(I != eI)[:5])
        assert bits_equal(D, eD)
    d = sets.row_query(77, [0, 529, 77, 300])
    _, eD = oracle.matrix(off, codes, 77, 78, 0, n)
    assert bits_equal(d, eD[0, [0, 529, 77, 300]])


@pytest.mark.parametrize("splits", [1, None])
def test_dense_tiles_mfma_past_f32_bound(ctx, opts, splits):
    """the FP4 MFMA tiles accumulate in f32, exact only
    for counts <= 2^24. Four near-identical 10 Mbp genomes (DNA k=21, both
    strands: ~20 M kmers each, GenomeProcessor.java:139-140's scale) share
    more than 2^24 dense kmers a pair; with one K split asked for (option
    bitset_mfma_splits 1) the launch must still split K so that no split
    sums more than 2^18 words, and I and D equal the oracle bit for bit
    (the raw-stage and nibble-operand MFMA tiles, and the AND + popcount
    tiles, option bitset_mfma 0)."""
    import gdist
    opts(sparse=0, bitset_mfma_splits=splits)
    n = 4
    seqs = synth_sets(n, 10_000_000, 0.001, 131)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    _, W = sets.build_bitsets(rare_threshold=0)
    assert W > (1 << 18), W                      # one split would pass the f32 bound
    off, codes = oracle_pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n, flags=0, nthreads=4)
    iu = np.triu_indices(n, 1)
    assert eI[iu].min() > (1 << 24), eI[iu]       # the premise: counts past 2^24
    for mfma, raw, km, plane in ((1, None, None, None), (1, None, None, 0), (1, None, 2, None), (1, 0, None, None),
                                 (0, None, None, None)):
        opts(bitset_mfma=mfma, bitset_mfma_raw=raw, bitset_mfma_km=km, bitset_mfma_plane=plane)
        for up in (True, False):
            I, D = sets.matrix(upper=up, method=gdist.METHOD_BITSET)
            if up:
                assert np.array_equal(I[iu], eI[iu]), (mfma, I[iu], eI[iu])
                assert bits_equal(D[iu], eD[iu])
            else:
                assert np.array_equal(I, eI), (mfma, I, eI)
                assert bits_equal(D, eD)


@pytest.mark.parametrize("fill", [None, 0, 5, 4, 1])
def test_fill_routes_on_sparse_sets(ctx, opts, fill):
    """C3-shaped proteomes (sets much smaller than the dictionary, T > N so
    the rare tier holds every shared kmer): the bitset fill by hash probes (the
    default for such sets: fill_sort absent, or 4), by LDS windows (0: its
    global-walk fallback) and by the sort (1) give the same bit-exact counts
    and distances as the oracle."""
    import gdist
    opts(fill_sort=fill)
    n = 300
    seqs = synth_sets(n, 1500, 0.10, 109, protein=True)
    sets = gdist.KmerSets.from_sequences(seqs, 8, gdist.KmerType.PROT, 0, ctx)
    sets.build_bitsets(rare_threshold=1000)
    assert sets.rare_info()[1] > 0
    off, codes = oracle_pack(seqs, 8, 1, 0)
    for (r0, r1, c0, c1, up) in [(0, n, 0, n, True), (41, 250, 7, 290, False)]:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
        eI, eD = oracle.matrix(off, codes, r0, r1, c0, c1, flags=0x100 if up else 0)
        if up:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI), (fill, r0, r1, c0, c1, up)
        assert bits_equal(D, eD)
    sets.build_bitsets(rare_threshold=3)          # dense tier + rare lists
    I, D = sets.matrix(upper=True, method=gdist.METHOD_BITSET)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n, flags=0x100)
    iu = np.triu_indices(n, 1)
    assert np.array_equal(I[iu], eI[iu]) and bits_equal(D[iu], eD[iu])


def test_auto_method_prepare(ctx):
    """METHOD_AUTO: small regions stay on the sorted join without building a
    dictionary; a large region of C3-like proteomes (two-tier structure) is
    costed and runs on bitsets; a diverse collection is costed and falls back
    to the sorted join (bitsets freed). Every route is bit-exact."""
    import gdist
    n = 240
    seqs = synth_sets(n, 4000, 0.10, 103, protein=True)
    off, codes = oracle_pack(seqs, 8, 1, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n)

    small = gdist.KmerSets.from_sequences(seqs, 8, gdist.KmerType.PROT, 0, ctx)
    m, cb, cs = small.prepare(gdist.METHOD_AUTO)        # sorted estimate ~0.3 ms < 20 ms
    assert m == gdist.METHOD_SORTED and cb == -1.0 and cs > 0
    assert small.bitset_info()[1] == 0

    sets = gdist.KmerSets.from_sequences(seqs, 8, gdist.KmerType.PROT, 0, ctx)
    m, cb, cs = sets.prepare(gdist.METHOD_AUTO, pairs=float(1 << 22))
    assert m == gdist.METHOD_BITSET and 0 < cb < cs
    thr, lists, recs = sets.rare_info()
    assert lists > 0
    I, D = sets.matrix(method=gdist.METHOD_AUTO)
    assert np.array_equal(I, eI) and bits_equal(D, eD)

    # unrelated random proteomes: nothing is shared, the dictionary is empty,
    # yet the model must not pick a path slower than the join; either way exact
    rnd = [bytes(np.random.default_rng(7 + i).choice(np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8), 4000))
           for i in range(n)]
    div = gdist.KmerSets.from_sequences(rnd, 8, gdist.KmerType.PROT, 0, ctx)
    m, cb, cs = div.prepare(gdist.METHOD_AUTO, pairs=float(1 << 22))
    assert (m == gdist.METHOD_BITSET) == (0 <= cb <= cs)
    roff, rcodes = oracle_pack(rnd, 8, 1, 0)
    rI, rD = oracle.matrix(roff, rcodes, 0, n, 0, n)
    I, D = div.matrix(method=gdist.METHOD_AUTO)
    assert np.array_equal(I, rI) and bits_equal(D, rD)


def test_single_rank_allgather_bitsets(ctx):
    """gdist_sets_allgather_bitsets without a communicator = one rank: same
    counts as the local build (exercises the distributed code path)."""
    import gdist
    seqs = synth_sets(150, 4000, 0.02, 102)
    local = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    ag = local.allgather_bitsets()
    I, D = ag.matrix(method=gdist.METHOD_BITSET)
    off, codes = oracle_pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, 150, 0, 150)
    assert np.array_equal(I, eI) and bits_equal(D, eD)
    with pytest.raises(ValueError):
        ag.matrix(method=gdist.METHOD_SORTED)          # bitset-only collection


def test_width_processor_vs_restatement(ctx):
    """WidthProcessor output (WidthProcessor.java:115-208) against a pure-Python
    restatement on pyref sets / sketches: same lines, bit for bit."""
    import gdist
    from gdist import processors as P
    from gdist.javafmt import java_format_f
    g1 = [bytes(r).decode() for r in __import__("gdist").synth.genomes(14, 300, 0.10, 107, protein=True)]
    g2 = [bytes(r).decode() for r in __import__("gdist").synth.genomes(11, 250, 0.30, 108, protein=True)]
    rows = [("fam1", s) for s in g1] + [("fam2", s) for s in g2]
    out = io.StringIO()
    target = P.width_processor(rows, 20, 60, out, step=20, max_group=12, target_error=0.05, kmer_size=8, ctx=ctx)
    # restatement: groups of <= 12 consecutive rows of one id
    exp, tgt = ["Group\tSize\tPairs\tDwarves\tMean E\tMax E"], 20
    groups, cur, gid = [], [], ""
    for g, s in rows:
        if g != gid or len(cur) >= 12:
            if cur:
                groups.append((gid, cur))
            gid, cur = g, []
        cur.append(s)
    groups.append((gid, cur))
    for gid, prots in groups:
        sets = [pyref.kmer_set(p, 8, pyref.PROT) for p in prots]
        n = len(sets)
        real = {(i, j): pyref.set_distance(sets[i], sets[j]) for i in range(n) for j in range(i + 1, n)}
        pairs = sum(1 for v in real.values() if v < 1.0)
        if not pairs:
            continue
        good = P.INVALID_TARGET_SIZE
        for size in (20, 40, 60):
            sk = [pyref.sketch(s, size) for s in sets]
            dwarves = sum(1 for x in sk if len(x) < size)
            total, mx = 0.0, 0.0
            for i in range(n):
                for j in range(i + 1, n):
                    sd = pyref.sketch_distance(sk[i], sk[j], size)[0]
                    r = real[(i, j)]
                    if r != sd:
                        e = abs(r - sd) * 2.0 / (r + sd)
                        mx = e if e > mx else mx
                        total += e
            mean = total / pairs
            exp.append(f"{gid}\t{size:8d}\t{pairs:8d}\t{dwarves:8d}\t{java_format_f(mean, 8, 4)}\t"
                       f"{java_format_f(mx, 8, 4)}")
            if size < good and mean <= 0.05:
                good = size
        tgt = max(tgt, good)
    assert out.getvalue().splitlines() == exp
    assert target == tgt


@pytest.mark.parametrize("sparse", [True, False])
def test_graph_replay_of_repeated_steps(ctx, opts, sparse):
    """Repeated matrix calls into the same device outputs replay the step as
    a hipGraph (option graph): the second call is captured, later calls
    launch the graph. Every call — including after the outputs were
    overwritten — equals the oracle, and equals the uncaptured path."""
    import gdist
    n = 300
    seqs = synth_sets(n, 20000, 0.003, 107)
    opts(sparse_zmax=100000 if sparse else None, sparse=None if sparse else 0)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    assert (sets.sparse_info()[0] > 0) == sparse
    # a rare tier: the replayed sparse step recounts its pairs every call (the
    # per-step slab is zeroed inside the graph; a stale slab would add them twice)
    assert sets.rare_info()[1] > 0
    off, codes = oracle_pack(seqs, 21, 0, 0)
    for (r0, r1) in [(0, n), (37, 211)]:
        eI, eD = oracle.matrix(off, codes, r0, r1, 0, n, flags=0x100)
        nr = r1 - r0
        dI, dD = ctx.alloc(nr * n * 4), ctx.alloc(nr * n * 8)
        mask = np.fromfunction(lambda a, b: b > (r0 + a), (nr, n))
        for call in range(4):
            dI.from_host(np.full(nr * n, -7, np.int32))
            dD.from_host(np.full(nr * n, 42.5))
            sets.matrix_device(dI.ptr, dD.ptr, n, (r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
            I = dI.to_host(np.int32).reshape(nr, n)
            D = dD.to_host(np.float64).reshape(nr, n)
            assert np.array_equal(I[mask], eI[mask]) and bits_equal(D[mask], eD[mask]), (r0, call)
            assert np.all(I[~mask] == -7), (r0, call)           # below the diagonal untouched
        dI.free(); dD.free()


def test_from_blob_equals_from_sequences(ctx):
    """KmerSets.from_blob (one buffer + offsets, as bytes, bytearray or a
    uint8 array; what bench.py packs from) gives the same collection as
    from_sequences: identical counts and distances."""
    import gdist
    seqs = synth_sets(40, 3000, 0.02, 77)
    seqs[5] = b""                                            # an empty sequence in the middle
    off = np.zeros(len(seqs) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    blob = b"".join(seqs)
    ref = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
    eI, eD = ref.matrix(method=gdist.METHOD_SORTED)
    for b in (blob, bytearray(blob), np.frombuffer(blob, dtype=np.uint8)):
        s = gdist.KmerSets.from_blob(b, off, 15, gdist.KmerType.DNA, 0, ctx)
        assert np.array_equal(s.sizes(), ref.sizes())
        I, D = s.matrix(method=gdist.METHOD_SORTED)
        assert np.array_equal(I, eI) and bits_equal(D, eD)


def test_append_extends_segment_index(ctx):
    """gdist_sets_append on a collection whose sorted-join segment index is
    built (the Java methods drop-in's genome cache): the new sets' index rows
    are added with the collection's splitters instead of rebuilding the index
    (ADVICE r5), so sets larger than every old one (longer segments), an
    empty one and one at a time all join exactly; the bitset path after the
    appends agrees (GenomeProcessor.java:140, MethodTableProcessor.java:275)."""
    import gdist
    seqs = synth_sets(12, 6000, 0.03, 131)
    extra = synth_sets(4, 30000, 0.03, 132) + [b""] + synth_sets(2, 3000, 0.05, 133)
    sets = gdist.KmerSets.from_sequences(seqs[:8], 21, gdist.KmerType.DNA, 0, ctx)
    sets.matrix(method=gdist.METHOD_SORTED)              # builds the segment index
    have = list(seqs[:8])
    for batch in ([seqs[8]], seqs[9:12], extra[:1], extra[1:5], extra[5:]):
        first = sets.append(batch)
        assert first == len(have)
        have += batch
        n = len(have)
        off, codes = oracle_pack(have, 21, 0, 0)
        eI, eD = oracle.matrix(off, codes, 0, n, 0, n)
        I, D = sets.matrix(method=gdist.METHOD_SORTED)
        assert np.array_equal(I, eI) and bits_equal(D, eD), n
        d = sets.row_query(n - 1, list(range(n)))
        assert bits_equal(d, eD[n - 1])
    I, D = sets.matrix(method=gdist.METHOD_BITSET)
    assert np.array_equal(I[np.triu_indices(len(have), 1)], eI[np.triu_indices(len(have), 1)])


@pytest.mark.parametrize("mode", [1, 0])
def test_distance_epilogue_modes(ctx, opts, mode):
    """The distance epilogue (the Java expression of SequenceKmers.distance,
    FastaDistanceProcessor.java:186) by rows (option epilogue_rows 1,
    default) and the flat kernel (0): bit-exact over upper triangles and
    rectangles whose rows start at every alignment, odd column counts, host
    and device outputs (poisoned first), with empty sets under both
    empty-set readings (GDIST_EMPTY_NAN). (Round 6 measured a four-column
    form slower on C3 — 1.54 vs 1.50 ms a step — and removed it.)"""
    import gdist
    opts(epilogue_rows=mode, sparse=0)                      # no fused sparse step: the epilogue kernels
    seqs = synth_sets(53, 3000, 0.04, 141)
    seqs[7] = b""
    seqs[30] = b"ACGT"                                          # shorter than k: empty
    off, codes = oracle_pack(seqs, 21, 0, 0)
    n = len(seqs)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    for flags in (0, 0x400):
        for (r0, r1, c0, c1, up) in [(0, n, 0, n, True), (1, 50, 3, 52, True), (5, 38, 2, 51, False),
                                     (30, 33, 0, n, False), (52, 53, 0, n, False)]:
            fl = flags | (0x100 if up else 0)
            eI, eD = oracle.matrix(off, codes, r0, r1, c0, c1, flags=fl)
            I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET, flags=flags)
            m = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0)) if up else \
                np.ones((r1 - r0, c1 - c0), bool)
            assert np.array_equal(I[m], eI[m]), (mode, flags, r0, r1, c0, c1)
            assert bits_equal(D[m], eD[m]), (mode, flags, r0, r1, c0, c1)
            # device outputs (the bench's form), poisoned first
            nr, nc = r1 - r0, c1 - c0
            dI, dD = ctx.alloc(nr * nc * 4), ctx.alloc(nr * nc * 8)
            dI.from_host(np.full(nr * nc, -7, np.int32))
            dD.from_host(np.full(nr * nc, 42.5))
            sets.matrix_device(dI.ptr, dD.ptr, nc, (r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET,
                               flags=flags)
            gI = dI.to_host(np.int32).reshape(nr, nc)
            gD = dD.to_host(np.float64).reshape(nr, nc)
            assert np.array_equal(gI[m], eI[m]) and bits_equal(gD[m], eD[m]), (mode, flags, r0, "device")
            dI.free(); dD.free()
