"""The variant tier (csrc/variant.hip) and the code-range
dictionary, bit-exact against the oracle.

C4's structure at a size the oracle checks quickly: one ancestor, genomes
with independent substitutions, many genomes per site so that every
single-substitution kmer is shared by several genomes (C4: ~500 of
100,000). Options force the tiers the full size would choose: kmers held by
>= variant_dmin sets are dense bit columns, by rare_t .. variant_dmin - 1
variant words (grouped by the substitution through their Hamming-1 dense
neighbour), by 2 .. rare_t - 1 posting lists. Reference loop:
FastaDistanceProcessor.java:157-186 (every pair of a row block).
"""
import numpy as np
import pytest

import oracle
import refcache

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a, np.float64).view(np.uint64),
                          np.ascontiguousarray(b, np.float64).view(np.uint64))


@pytest.fixture(scope="module")
def c4_like():
    from gdist import synth
    n = 1200
    seqs = [bytes(r) for r in synth.genomes(n, 4000, 0.03, 41)]
    off, codes = oracle.pack(seqs, 21, 0, 0)
    return seqs, off, codes


REGIONS = [(0, 1200, 0, 1200, True), (37, 211, 5, 1190, False), (600, 1200, 0, 1200, True),
           (1199, 1200, 0, 1200, False)]


@pytest.mark.parametrize("mode", ["variant", "variant_windowed_fill", "variant_w64", "variant_unpacked", "variant_store",
                                  "variant_keyless_rare", "variant_keyless_words", "variant_key1", "range_only",
                                  "two_tier"])
def test_variant_tier_exact(ctx, opts, c4_like, mode):
    """Counts and distances of the variant tier (its hash fill and the
    windowed fill; 47-kmer words of 8-byte packed members (default), 64-kmer
    words (option variant_bits 64), the packed words walked from the 4 +
    8-byte arrays (variant_short 0); the code-range dictionary alone; the two
    tiers) equal the oracle's over upper triangles, rectangles, unaligned row
    blocks and row queries; the grouping puts each substitution's kmers into
    one word (words << kmers)."""
    import gdist
    seqs, off, codes = c4_like
    n = len(seqs)
    if mode == "two_tier":
        opts(variant=0, rare_t=3)
    elif mode == "range_only":
        opts(variant=0, rare_t=3, range_summary=1)
    else:
        # the hash fill (default) or the two-tier build's windowed fill (fill_sort 3)
        opts(variant=1, rare_t=3, variant_dmin=n // 10, range_summary=1,
             fill_sort=3 if mode == "variant_windowed_fill" else None,
             variant_bits=64 if mode == "variant_w64" else None,
             variant_short=0 if mode == "variant_unpacked" else None,
             bitset_mfma_store=1 if mode == "variant_store" else None,
             # round 6: keyless kmers as rare posting lists (forced) or words
             variant_keyless_rare={"variant_keyless_rare": 1, "variant_keyless_words": 0}.get(mode),
             # round 6: second-level keys (default) or the first level only
             variant_key2=0 if mode == "variant_key1" else None)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    vk, vw, ve, vp = sets.variant_info()
    if mode.startswith("variant"):
        assert vk > 1000 and ve > 0 and vp > 0, (vk, vw, ve, vp)
        assert vw * 8 < vk, ("substitution grouping", vk, vw)
        wk, mb, _ = sets.variant_layout()
        assert (wk, mb) == ((64, 12) if mode == "variant_w64" else (47, 8)), (mode, wk, mb)
    else:
        assert (vk, vw, ve) == (0, 0, 0)
    for (r0, r1, c0, c1, up) in REGIONS:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
        eI, eD = refcache.matrix(off, codes, r0, r1, c0, c1, flags=0x100 if up else 0, nthreads=8)
        if up:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI), (mode, r0, r1, c0, c1, up, np.flatnonzero(I != eI)[:5])
        assert bits_equal(D, eD)
    cols = [4, n - 1, 0, 600, 600, 17]
    d = sets.row_query(600, cols)
    _, eD = refcache.matrix(off, codes, 600, 601, 0, n)
    assert bits_equal(d, eD[0, cols])


def test_rebuild_drops_variant_tier(ctx, opts, c4_like):
    """a collection built with the variant tier and then
    rebuilt without it (option variant 0, another rare threshold, or kept
    singletons) must not keep the old variant lists: every rebuild equals
    the oracle, and variant_info reports the new tiers only."""
    import gdist
    seqs, off, codes = c4_like
    n = len(seqs)
    opts(variant=1, rare_t=3, variant_dmin=n // 10)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    assert sets.variant_info()[0] > 0
    r0, r1 = 300, 700
    eI, eD = refcache.matrix(off, codes, r0, r1, 0, n, flags=0x100, nthreads=8)
    mask = np.fromfunction(lambda a, b: b > (r0 + a), (r1 - r0, n))

    def check(tag):
        I, D = sets.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
        assert np.array_equal(I[mask], eI[mask]), (tag, np.flatnonzero(I[mask] != eI[mask])[:5])
        assert bits_equal(D[mask], eD[mask]), tag
        d = sets.row_query(500, [0, 17, n - 1, 500])
        assert bits_equal(d, refcache.matrix(off, codes, 500, 501, 0, n)[1][0, [0, 17, n - 1, 500]]), tag

    check("variant")
    opts(variant=0)
    sets.build_bitsets()                          # two tiers, same rare_t
    assert sets.variant_info()[:3] == (0, 0, 0)
    check("two-tier rebuild")
    opts(variant=1)
    sets.build_bitsets()
    assert sets.variant_info()[0] > 0
    check("variant again")
    opts(variant=None, rare_t=None)
    sets.build_bitsets(rare_threshold=5)          # a given threshold
    check("rare_t 5")
    sets.build_bitsets(keep_singletons=True)
    assert sets.variant_info()[:3] == (0, 0, 0)
    check("keep singletons")


def test_variant_tier_replayed_steps(ctx, opts, c4_like):
    """Repeated device-output calls (plan, capture, replay) of a variant-tier
    collection: every call equals the oracle (the variant walk's atomics land
    on a zeroed region each step)."""
    import gdist
    seqs, off, codes = c4_like
    n = len(seqs)
    opts(variant=1, rare_t=3, variant_dmin=n // 10)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    assert sets.variant_info()[0] > 0
    r0, r1 = 100, 400
    eI, eD = refcache.matrix(off, codes, r0, r1, 0, n, flags=0x100, nthreads=8)
    nr = r1 - r0
    dI, dD = ctx.alloc(nr * n * 4), ctx.alloc(nr * n * 8)
    mask = np.fromfunction(lambda a, b: b > (r0 + a), (nr, n))
    for call in range(4):
        sets.matrix_device(dI.ptr, dD.ptr, n, (r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
        I = dI.to_host(np.int32).reshape(nr, n)
        D = dD.to_host(np.float64).reshape(nr, n)
        assert np.array_equal(I[mask], eI[mask]) and bits_equal(D[mask], eD[mask]), call
    dI.free()
    dD.free()


POISON_CASES = {
    # the grouped rare tier (variant_short_kernel) beside the raw-stage MFMA
    # tiles (c4_like's ~125 dense words >= 64): 16-bit counters, one slice a row
    "grouped_dna": ("c4", dict(variant=0, rare_group=1)),
    # ... 32-bit counters, two slices a row
    "grouped_dna_c32_split2": ("c4", dict(variant=0, rare_group=1, variant_c16=0, variant_split=2)),
    # C3's shape (protein k=8): the short walk beside the AND + popcount tiles
    "grouped_protein": ("c3", dict(variant=0, rare_group=1)),
    # C4's variant walk (variant_rows_kernel, 8-byte members) + MFMA tiles +
    # the row-major rare walk in LDS column chunks ...
    "variant": ("c4", dict(variant=1, rare_t=3, variant_dmin=120)),
    # ... or by rare_rows_direct_kernel (atomics into I)
    "variant_direct": ("c4", dict(variant=1, rare_t=3, variant_dmin=120, rare_direct=1)),
}


@pytest.mark.parametrize("case", list(POISON_CASES))
def test_replayed_steps_poisoned(ctx, opts, c3_like, c4_like, case):
    """repeated device-output calls over one region (the
    first runs uncaptured and builds the plans, the second is captured, the
    rest replay the hipGraph) into outputs POISONED before every call (I =
    -7, D = 42.5): a replayed graph that dropped a kernel family's launch, or
    the zeroing, would leave poison or miss that family's counts. Every call
    equals the oracle over the region's upper triangle
    (FastaDistanceProcessor.java:177-186: each row block's pairs)."""
    import gdist
    data, o = POISON_CASES[case]
    seqs, off, codes = c3_like if data == "c3" else c4_like
    kind, k = (gdist.KmerType.PROT, 8) if data == "c3" else (gdist.KmerType.DNA, 21)
    n = len(seqs)
    opts(**o)
    sets = gdist.KmerSets.from_sequences(seqs, k, kind, 0, ctx)
    sets.build_bitsets()
    vk, vw, ve, _ = sets.variant_info()
    assert vk > 0 and ve > 0, (case, vk, ve)
    if case.startswith("grouped"):
        assert sets.variant_layout()[:2] == (16, 4) and sets.rare_info()[1] == 0, case
    else:
        assert sets.variant_layout()[:2] == (47, 8) and sets.rare_info()[1] > 0, case
    if data == "c4":
        assert sets.bitset_info()[1] >= 64, "the dense tiles run on the matrix cores"
    for (r0, r1) in [(0, n), (100, 400)]:
        nr = r1 - r0
        eI, eD = refcache.matrix(off, codes, r0, r1, 0, n, flags=0x100)
        mask = np.fromfunction(lambda a, b: b > (r0 + a), (nr, n))
        dI, dD = ctx.alloc(nr * n * 4), ctx.alloc(nr * n * 8)
        pI, pD = np.full(nr * n, -7, np.int32), np.full(nr * n, 42.5)
        for call in range(4):
            dI.from_host(pI)
            dD.from_host(pD)
            sets.matrix_device(dI.ptr, dD.ptr, n, (r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
            I = dI.to_host(np.int32).reshape(nr, n)
            D = dD.to_host(np.float64).reshape(nr, n)
            assert np.array_equal(I[mask], eI[mask]), (case, r0, call, np.flatnonzero(I[mask] != eI[mask])[:5])
            assert bits_equal(D[mask], eD[mask]), (case, r0, call)
        dI.free()
        dD.free()


def test_variant_greedy_reps(ctx, opts, c4_like):
    """Greedy representatives (DistanceRepsProcessor.java:185-262) over a
    variant-tier collection: the device's reps and assignments follow the
    oracle's distances."""
    import gdist
    seqs, off, codes = c4_like
    n = 300
    opts(variant=1, rare_t=3, variant_dmin=30)
    sets = gdist.KmerSets.from_sequences(seqs[:n], 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    assert sets.variant_info()[0] > 0
    o2, c2 = oracle.pack(seqs[:n], 21, 0, 0)
    _, eD = oracle.matrix(o2, c2, 0, n, 0, n, nthreads=8)
    t = float(np.quantile(eD[np.triu_indices(n, 1)], 0.02))
    is_rep, rep_of, rep_d = sets.greedy_reps(t, assign=True)
    reps = []
    for i in range(n):
        if not any(eD[i, r] <= t for r in reps):
            reps.append(i)
    assert list(np.flatnonzero(is_rep)) == reps
    for i in range(n):
        if not is_rep[i]:
            assert rep_d[i] == min(eD[i, r] for r in reps)


def test_variant_walk_across_column_chunks(ctx, opts):
    """The variant row walk counts a row against its columns in LDS chunks
    (32,768 columns of 16-bit counters; 16,384 of 32-bit) and keeps each list's position from chunk to chunk (C4:
    100,000 columns, 7 chunks); round 5 loads the next 64 members of a list
    before counting the current ones. 17,000 sets: rows whose lists cross
    chunk boundaries, both rare walks (LDS chunks and direct atomics), equal
    the oracle."""
    import gdist
    from gdist import synth
    n = 17000
    seqs = [bytes(r) for r in synth.genomes(n, 600, 0.03, 43)]
    off, codes = oracle.pack(seqs, 21, 0, 0)
    opts(variant=1, rare_t=3, variant_dmin=n // 10, range_summary=1)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    vk, vw, ve, vp = sets.variant_info()
    assert vk > 0 and ve > 0, (vk, vw, ve)
    for direct, c16, split in ((None, None, None), (0, 0, None), (1, None, 1), (None, 0, 3)):
        # option variant_c16 (default): 16-bit counters in 32,768-column
        # chunks (0: 32-bit in 16,384); variant_split: slices a row
        opts(rare_direct=direct, variant_c16=c16, variant_split=split)
        for (r0, r1, up) in [(0, 24, True), (16370, 16400, True), (500, 520, False), (0, 8, False)]:
            I, D = sets.matrix((r0, r1), (0, n), upper=up, method=gdist.METHOD_BITSET)
            eI, eD = oracle.matrix(off, codes, r0, r1, 0, n, flags=0x100 if up else 0, nthreads=8)
            if up:
                mask = np.fromfunction(lambda a, b: b > (r0 + a), (r1 - r0, n))
                I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
            assert np.array_equal(I, eI), (direct, c16, split, r0, r1, np.flatnonzero(I != eI)[:5])
            assert bits_equal(D, eD), (direct, r0, r1)


@pytest.fixture(scope="module")
def c3_like():
    """C3's structure (one ancestral proteome, independent substitutions, a
    few sets a substitution) at 1,500 x 3,000 aa."""
    from gdist import synth
    n = 1500
    seqs = [bytes(r) for r in synth.genomes(n, 3000, 0.10, 45, protein=True)]
    off, codes = oracle.pack(seqs, 8, 1, 0)
    return seqs, off, codes


@pytest.mark.parametrize("data,walk", [("protein", "short"), ("protein", "short_c32"), ("protein", "short_split"),
                                       ("protein", "wave"), ("protein", "store"), ("protein", "own_words"),
                                       ("dna", "short"), ("dna", "wave")])
def test_grouped_rare_tier_exact(ctx, opts, c3_like, c4_like, data, walk):
    """Round 5, option rare_group: the kmers of 2 .. T - 1 sets as 16-kmer
    variant words (one substitution a word; DNA's 42 kmers of a substitution
    in three) walked a thread an entry over packed (set | mask << 16) lists,
    16-bit (default) or 32-bit LDS counters, several slices a row, or by the
    wave-per-entry walk; counts and distances equal the oracle's over upper
    triangles, rectangles, unaligned row blocks and row queries, and the rare
    posting tier is empty."""
    import gdist
    seqs, off, codes = c3_like if data == "protein" else c4_like
    n = len(seqs)
    opts(variant=0, rare_group=1, variant_short=0 if walk == "wave" else None,
         variant_c16=0 if walk == "short_c32" else None, variant_split=3 if walk == "short_split" else None,
         bitset_mfma_store=1 if walk == "store" else None, variant_pack_keyless=0 if walk == "own_words" else None)
    kind, k = (gdist.KmerType.PROT, 8) if data == "protein" else (gdist.KmerType.DNA, 21)
    sets = gdist.KmerSets.from_sequences(seqs, k, kind, 0, ctx)
    sets.build_bitsets()
    vk, vw, ve, vp = sets.variant_info()
    thr, lists, recs = sets.rare_info()
    assert vk > 1000 and ve > 0 and lists == 0 and thr == 2, (vk, vw, ve, thr, lists)
    assert vw * 3 < vk, ("substitution grouping", vk, vw)
    wk, mb, wmax = sets.variant_layout()
    assert wk == 16 and mb == 4 and 0 < wmax < 65536, (wk, mb, wmax)
    for (r0, r1, c0, c1, up) in [(0, n, 0, n, True), (37, 211, 5, n - 10, False), (n // 2, n, 0, n, True),
                                 (n - 1, n, 0, n, False)]:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
        eI, eD = refcache.matrix(off, codes, r0, r1, c0, c1, flags=0x100 if up else 0, nthreads=8)
        if up:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI), (data, walk, r0, r1, c0, c1, up, np.flatnonzero(I != eI)[:5])
        assert bits_equal(D, eD)
    cols = [4, n - 1, 0, 600, 600, 17]
    d = sets.row_query(600, cols)
    _, eD = refcache.matrix(off, codes, 600, 601, 0, n)
    assert bits_equal(d, eD[0, cols])


def test_grouped_rare_tier_keyless(ctx, opts, c3_like):
    """Without locus keys (no guide sequences: option guides 0) every rare
    kmer is keyless. A probing grouped build (the default choice; option
    rare_group 2) then keeps the two tiers; a forced one (rare_group 1) gives
    each keyless kmer a word of its own instead of packing unrelated kmers
    into one list. Both equal the oracle."""
    import gdist
    seqs, off, codes = c3_like
    n = len(seqs)
    eI, eD = refcache.matrix(off, codes, 0, n, 0, n, flags=0x100, nthreads=8)
    iu = np.triu_indices(n, 1)
    for rg in (2, 1):
        opts(variant=None, rare_group=rg, guides=0)
        sets = gdist.KmerSets.from_sequences(seqs, 8, gdist.KmerType.PROT, 0, ctx)
        sets.build_bitsets()
        vk, vw, ve, _ = sets.variant_info()
        thr, lists, _ = sets.rare_info()
        if rg == 2:
            assert vk == 0 and lists > 0 and thr > 2, (vk, thr, lists)
        else:
            assert vk > 0 and vw == vk and lists == 0, ("a word each", vk, vw, lists)
        I, D = sets.matrix(upper=True, method=gdist.METHOD_BITSET)
        assert np.array_equal(I[iu], eI[iu]), (rg, np.flatnonzero(I[iu] != eI[iu])[:5])
        assert bits_equal(D[iu], eD[iu]), rg


def test_grouped_rare_walk_across_column_chunks(ctx, opts):
    """The short-list walk over 17,000 columns: two 16,384-column LDS chunks,
    rows whose lists cross the boundary, equal the oracle."""
    import gdist
    from gdist import synth
    n = 17000
    seqs = [bytes(r) for r in synth.genomes(n, 600, 0.03, 43)]
    off, codes = oracle.pack(seqs, 21, 0, 0)
    opts(variant=0, rare_group=1)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    vk, vw, ve, vp = sets.variant_info()
    assert vk > 0 and ve > 0 and sets.rare_info()[1] == 0, (vk, vw, ve)
    for c16 in (None, 0):
        opts(variant_c16=c16)
        for (r0, r1, up) in [(0, 24, True), (16370, 16400, True), (500, 520, False)]:
            I, D = sets.matrix((r0, r1), (0, n), upper=up, method=gdist.METHOD_BITSET)
            eI, eD = oracle.matrix(off, codes, r0, r1, 0, n, flags=0x100 if up else 0, nthreads=8)
            if up:
                mask = np.fromfunction(lambda a, b: b > (r0 + a), (r1 - r0, n))
                I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
            assert np.array_equal(I, eI), (c16, r0, r1, np.flatnonzero(I != eI)[:5])
            assert bits_equal(D, eD), (c16, r0, r1)


@pytest.mark.parametrize("mode", ["variant", "variant_windowed_fill", "variant_keyless_rare", "two_tier",
                                  "two_tier_sort_fill"])
def test_split_build_equals_whole_build(ctx, opts, c4_like, mode):
    """the build of a gathered collection split by rank.
    Option split_build = 3 runs the three ranks' shares in turn on this GPU
    (share r: 1/3 of the summary's code ranges, the fill of sets [400 r,
    400 (r + 1))) and concatenates what the all-gathers would: the bitsets,
    tiers and counts equal the one-share build's and the oracle's."""
    import gdist
    seqs, off, codes = c4_like
    n = len(seqs)
    if mode.startswith("variant"):
        base = dict(variant=1, rare_t=3, variant_dmin=n // 10, range_summary=1,
                    fill_sort=3 if mode == "variant_windowed_fill" else None,
                    variant_keyless_rare=1 if mode == "variant_keyless_rare" else None)
    else:
        base = dict(variant=0, rare_t=3, fill_sort=1 if mode == "two_tier_sort_fill" else None)
    built = {}
    for split in (None, 3):
        opts(split_build=split, **base)
        sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
        sets.build_bitsets()
        bt = sets.build_timing()
        assert bt["shares"] == (split or 1), bt
        assert 0 <= bt["share_max_ms"] <= bt["split_ms"] <= bt["build_ms"], bt
        built[split] = (sets.bitsets(), sets.variant_info(), sets.rare_info(), sets)
    (b0, v0, r0_, _), (b3, v3, r3, s3) = built[None], built[3]
    assert np.array_equal(b0, b3) and v0 == v3 and r0_ == r3, (mode, v0, v3, r0_, r3)
    for (a, b, c0, c1, up) in REGIONS[:2]:
        I, D = s3.matrix((a, b), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
        eI, eD = refcache.matrix(off, codes, a, b, c0, c1, flags=0x100 if up else 0, nthreads=8)
        if up:
            mask = np.fromfunction(lambda x, y: (c0 + y) > (a + x), (b - a, c1 - c0))
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI), (mode, a, b)
        assert bits_equal(D, eD)


def test_release_codes(ctx, opts, c4_like):
    """gdist_sets_release_codes: a built collection drops its codes and keeps
    answering bitset calls (the C4 ranks' 160 GB of gathered codes); calls that
    need codes refuse it."""
    import gdist
    seqs, off, codes = c4_like
    n = len(seqs)
    opts(variant=1, rare_t=3, variant_dmin=n // 10)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    fresh = gdist.KmerSets.from_sequences(seqs[:5], 21, gdist.KmerType.DNA, 0, ctx)
    with pytest.raises(ValueError):
        fresh.release_codes()                      # no bitsets: the codes are all it has
    sets.build_bitsets()
    sets.release_codes()
    I, D = sets.matrix((0, 50), (0, n), upper=True, method=gdist.METHOD_AUTO)
    eI, eD = refcache.matrix(off, codes, 0, 50, 0, n, flags=0x100, nthreads=8)
    mask = np.fromfunction(lambda a, b: b > a, (50, n))
    assert np.array_equal(I[mask], eI[mask]) and bits_equal(D[mask], eD[mask])
    for call in (lambda: sets.matrix((0, 5), (0, n), method=gdist.METHOD_SORTED),
                 lambda: sets.build_bitsets(),
                 lambda: sets.download()):
        with pytest.raises(ValueError):
            call()
