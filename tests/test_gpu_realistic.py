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
