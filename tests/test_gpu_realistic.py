"""The locus order and the complement-/positive-sparse words beyond the
generator they were tuned on: genomes in clades with
short indels and segment moves / inversions (gdist.synth.realistic_genome),
whose guides are ordinary clade members. Counts and distances are bit-exact
against the CPU oracle with the sparse split as the cost model picks it,
forced on, and off; the model's choice is reported."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a, np.float64).view(np.uint64),
                          np.ascontiguousarray(b, np.float64).view(np.uint64))


@pytest.mark.parametrize("mode", ["model", "forced", "off"])
def test_realistic_collection_exact(ctx, opts, mode):
    import gdist
    from gdist import synth
    n = 160
    seqs = synth.realistic_genomes(n, 150_000, 0.002, 7, p_rearrange=0.7)
    assert len({len(s) for s in seqs}) > 1                    # indels: lengths differ
    opts(**{"model": {}, "forced": {"sparse_zmax": 100000}, "off": {"sparse": 0}}[mode])
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    ws, wd, ent = sets.sparse_info()
    cw, pw = sets.sparse_sides()
    print(f"realistic {mode}: sparse words {ws} ({cw} complement, {pw} positive), dense {wd}, entries {ent}, "
          f"rare {sets.rare_info()}")
    if mode == "forced":
        assert ws > 0
    if mode == "off":
        assert ws == 0
    off, codes = oracle.pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n, flags=0x100, nthreads=8)
    I, D = sets.matrix(upper=True, method=gdist.METHOD_BITSET)
    iu = np.triu_indices(n, 1)
    assert np.array_equal(I[iu], eI[iu]) and bits_equal(D[iu], eD[iu])
    for (r0, r1) in [(0, 37), (37, 101), (101, 160)]:           # row blocks as ranks get them
        Ib, _ = sets.matrix((r0, r1), (0, n), upper=True, method=gdist.METHOD_BITSET)
        mask = np.fromfunction(lambda a, b: b > (r0 + a), (r1 - r0, n))
        assert np.array_equal(Ib[mask], eI[r0:r1][mask]), (r0, r1)


@pytest.mark.parametrize("groups", [True, False])
def test_realistic_group_tier_exact(ctx, opts, groups):
    """The group tier on a clade-structured collection (8 clades of 50): the
    clade-variant words keep per member only its residual and the clade part
    is precomputed per pair (X); counts and distances bit-exact against the
    oracle, equal to the run without the tier (option sparse_groups = 0), over
    the whole triangle, rectangles and row blocks."""
    import gdist
    from gdist import synth
    n = 400
    seqs = synth.realistic_genomes(n, 60_000, 0.002, 9, p_rearrange=0.5)
    opts(sparse_groups=None if groups else 0)
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    ng, gw = sets.group_info()
    print(f"group tier {groups}: {ng} groups, {gw} words; sparse {sets.sparse_info()}")
    if groups:
        assert ng >= 4 and gw > 0
    else:
        assert ng == 0 and gw == 0
    off, codes = oracle.pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n, nthreads=8)
    iu = np.triu_indices(n, 1)
    I, D = sets.matrix(upper=True, method=gdist.METHOD_BITSET)
    assert np.array_equal(I[iu], eI[iu]) and bits_equal(D[iu], eD[iu])
    for (r0, r1, c0, c1, up) in [(0, n, 0, n, False), (37, 290, 11, 399, False), (130, 259, 0, n, True)]:
        Ib, Db = sets.matrix((r0, r1), (c0, c1), upper=up, method=gdist.METHOD_BITSET)
        E, ED = eI[r0:r1, c0:c1], eD[r0:r1, c0:c1]
        if up:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            Ib, Db, E, ED = Ib[mask], Db[mask], E[mask], ED[mask]
        assert np.array_equal(Ib, E) and bits_equal(Db, ED), (r0, r1, c0, c1, up)
    for mode in ({"sparse_fused": 0}, {"sparse_part_budget": 0, "sparse_chunks": 3}):
        opts(**mode)
        I2, _ = sets.matrix(upper=True, method=gdist.METHOD_BITSET)
        assert np.array_equal(I2[iu], eI[iu]), mode


_TWINS = {}


def _twin(kind):
    """The realistic C3 / C4 twins at a size the oracle checks quickly, with
    the oracle's whole matrix (tests/refcache.py): proteomes and 100 kbp-
    shaped genomes in 8 clades with indels and segment moves."""
    import refcache
    from gdist import synth
    if kind not in _TWINS:
        if kind == "c3r":
            seqs = synth.realistic_genomes(1500, 3000, 0.10, 45, protein=True, p_clade=0.01, indel_rate=2e-4)
            off, codes = oracle.pack(seqs, 8, 1, 0)
        else:
            seqs = synth.realistic_genomes(1200, 4000, 0.03, 41, p_clade=0.004, indel_rate=2e-4)
            off, codes = oracle.pack(seqs, 21, 0, 0)
        _TWINS[kind] = (seqs, off, codes, refcache.full(off, codes))
    return _TWINS[kind]


@pytest.mark.parametrize("twin,mode", [("c3r", "auto"), ("c3r", "grouped"), ("c3r", "two_tier"),
                                       ("c4r", "auto"), ("c4r", "variant"), ("c4r", "variant_direct"),
                                       ("c4r", "keyless_rare"), ("c4r", "keyless_words"), ("c4r", "key1"),
                                       ("c4r", "variant_dmin_default"),
                                       ("c3r", "grouped_key1")])
def test_realistic_twins_exact(ctx, opts, twin, mode):
    """C3's grouped rare tier (rare kmers as 16-kmer
    variant words keyed by their substitution site) and C4's variant tier off
    the star phylogeny — proteomes / genomes in clades, with indels (windows
    shift, so fewer kmers have a keyed dense neighbour) and segment moves:
    METHOD_AUTO's choice, the forced tiers and the two-tier fallback are all
    bit-exact against the oracle over upper triangles, row blocks and
    rectangles (GenomeProcessor.java:25-26, FastaDistanceProcessor.java:177-186)."""
    import gdist
    seqs, off, codes, (fI, fD) = _twin(twin)
    n = len(seqs)
    o = {"auto": {}, "grouped": dict(variant=0, rare_group=1), "two_tier": dict(variant=0, rare_group=0),
         "variant": dict(variant=1, rare_t=3, variant_dmin=n // 10),
         "variant_direct": dict(variant=1, rare_t=3, variant_dmin=n // 10, rare_direct=1),
         # round 6: the keyless kmers (segment-move junctions, windows across
         # indels) as rare posting lists, forced, or packed into words
         "keyless_rare": dict(variant=1, rare_t=3, variant_dmin=n // 10, variant_keyless_rare=1),
         "keyless_words": dict(variant=1, rare_t=3, variant_dmin=n // 10, variant_keyless_rare=0),
         # the first-level keys only (option variant_key2 = 0)
         "key1": dict(variant=1, rare_t=3, variant_dmin=n // 10, variant_key2=0),
         "variant_dmin_default": dict(variant=1, rare_t=3),             # Dmin = N / 20 (round 6)
         "grouped_key1": dict(variant=0, rare_group=1, variant_key2=0)}[mode]
    opts(**o)
    kind, k = (gdist.KmerType.PROT, 8) if twin == "c3r" else (gdist.KmerType.DNA, 21)
    assert len({len(s) for s in seqs}) > 1                    # indels: lengths differ
    sets = gdist.KmerSets.from_sequences(seqs, k, kind, 0, ctx)
    if mode == "auto":
        m, cb, cs = sets.prepare(gdist.METHOD_AUTO)
        method = gdist.METHOD_AUTO
    else:                                                   # the tiers built whatever AUTO would price
        sets.build_bitsets()
        m, cb, cs = sets.prepare(gdist.METHOD_BITSET)
        method = gdist.METHOD_BITSET
    vk, vw, ve, _ = sets.variant_info()
    print(f"{twin} {mode}: AUTO -> {m} (bitset {cb:.3g} s, sorted {cs:.3g} s), variant {vk} kmers "
          f"{vw} words {ve} entries, rare {sets.rare_info()}")
    if mode in ("grouped", "variant", "variant_direct", "keyless_rare", "keyless_words", "key1", "grouped_key1",
                "variant_dmin_default"):
        assert vk > 0 and ve > 0, (twin, mode, vk, ve)
        assert vw < vk, ("kmers grouped into words", vk, vw)
    if mode == "two_tier":
        assert vk == 0
    for (r0, r1, c0, c1, up) in [(0, n, 0, n, True), (100, 400, 0, n, True), (37, 211, 5, n - 10, False)]:
        I, D = sets.matrix((r0, r1), (c0, c1), upper=up, method=method)
        eI, eD = fI[r0:r1, c0:c1], fD[r0:r1, c0:c1]
        if up:
            mask = np.fromfunction(lambda a, b: (c0 + b) > (r0 + a), (r1 - r0, c1 - c0))
            I, D, eI, eD = I[mask], D[mask], eI[mask], eD[mask]
        assert np.array_equal(I, eI), (twin, mode, r0, r1, np.flatnonzero(I != eI)[:5])
        assert bits_equal(D, eD), (twin, mode, r0, r1)
