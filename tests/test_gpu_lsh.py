"""LSH bucket query on the device (gdist_lsh_build / gdist_lsh_closest):
getClosest(kmers, n, maxDist) of MashProcessor.java:150 / FindProcessor.java:110
against the oracle's restatement of the same bucket search (oracle.lsh_closest):
identical targets, order and fp64 distances. Parity with the reference's LSH
classes is unpinned (un-vendored org.theseed:sequence)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stages,buckets", [(15, 100), (4, 7), (1, 1)])
def test_lsh_closest_vs_oracle(ctx, stages, buckets):
    import gdist
    from gdist import synth
    subj = [bytes(r) for r in synth.genomes(300, 8000, 0.08, 31)]
    extra = [bytes(r) for r in synth.genomes(20, 8000, 0.08, 31, first=300)]
    width = 200
    S = gdist.KmerSets.from_sequences(subj, 21, gdist.KmerType.DNA, 0, ctx).sketches(width)
    Q = gdist.KmerSets.from_sequences(subj[:10] + extra, 21, gdist.KmerType.DNA, 0, ctx).sketches(width)
    so, sv = S.download()
    qo, qv = Q.download()
    ssig = [sv[so[i]:so[i + 1]] for i in range(len(so) - 1)]
    qsig = [qv[qo[i]:qo[i + 1]] for i in range(len(qo) - 1)]
    idx = gdist.LSHIndex(S, stages, buckets, seed=77)
    for n, md in ((10, 0.9), (3, 0.5), (50, 1.0)):
        got = idx.getClosest(Q, n, md)
        exp = oracle.lsh_closest(ssig, qsig, width, stages, buckets, 77, n, md)
        assert got == exp, (n, md)
    # a subject queried against its own index finds itself at distance 0 first
    got = idx.getClosest(Q, 1, 0.9)
    assert [g[0] for g in got[:10]] == [(i, 0.0) for i in range(10)]
    idx.free()
