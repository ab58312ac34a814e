"""Worker of tests/test_gpu_rccl.py: RCCL itself on one GPU. A one-rank
communicator (ncclCommInitRank, gdist_comm_init) with option force_exchange
runs every collective of the exchange paths (ncclAllGather of offsets, codes,
signatures, dictionary summaries, locus keys, bitsets, sizes and rare
records); the gathered collections must give the oracle's counts."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gdist  # noqa: E402
import oracle  # noqa: E402  (test infrastructure: the checker)
from gdist import synth  # noqa: E402


def main():
    ctx = gdist.Context(0)
    ctx.comm_init(gdist.Context.unique_id(), 1, 0)
    ctx.set_option("force_exchange", 1)
    assert ctx.allreduce_max(3.5) == 3.5
    n = 200
    seqs = [bytes(r) for r in synth.genomes(n, 100_000, 0.002, 21)]
    local = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    off, codes = oracle.pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n, flags=0x100, nthreads=8)
    iu = np.triu_indices(n, 1)
    ctx.set_option("sparse_zmax", 100000)            # the locus-key exchange + sparse words
    gb = local.allgather_bitsets()
    assert gb.sparse_info()[0] > 0
    I, D = gb.matrix(upper=True, method=gdist.METHOD_BITSET)
    assert np.array_equal(I[iu], eI[iu]) and np.array_equal(D[iu].view(np.uint64), eD[iu].view(np.uint64))
    gs = local.allgather()
    I, D = gs.matrix(upper=True, method=gdist.METHOD_SORTED)
    assert np.array_equal(I[iu], eI[iu]) and np.array_equal(D[iu].view(np.uint64), eD[iu].view(np.uint64))
    # the in-place code all-gather that consumes its shard (C4's exchange)
    own = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    gc = own.allgather(consume=True)
    del own
    I, D = gc.matrix(upper=True, method=gdist.METHOD_SORTED)
    assert np.array_equal(I[iu], eI[iu]) and np.array_equal(D[iu].view(np.uint64), eD[iu].view(np.uint64))
    assert [a.tolist() for a in gc.download()] == [off.tolist(), codes.tolist()]
    sk = local.sketches(100)
    ska = sk.allgather()
    assert [a.tolist() for a in ska.download()] == [a.tolist() for a in sk.download()]
    C1, D1 = sk.matrix(upper=True)
    C2, D2 = ska.matrix(upper=True)
    assert np.array_equal(C1[iu], C2[iu]) and np.array_equal(D1[iu].view(np.uint64), D2[iu].view(np.uint64))
    ctx.comm_destroy()
    print("RCCL_OK", flush=True)


if __name__ == "__main__":
    main()
