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
