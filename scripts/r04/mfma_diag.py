"""The k=32 all-ones-code case (tests/test_gpu_parity.py::test_k32_all_ones_code)
with singletons kept, through the MFMA and the AND+popcount dense tiles:
sizes, tiers and the pairs that differ from the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gdist  # noqa: E402
import oracle  # noqa: E402

rng = np.random.default_rng(111)
seqs = []
for i in range(24):
    body = "".join(rng.choice(list("ACGT"), 300))
    seqs.append((body[:150] + ("T" * 40 if i % 3 else "") + body[150:] + ("A" * 33 if i % 4 == 0 else "")).encode())
ctx = gdist.Context(0)
for strand in (1,):
    off, codes = oracle.pack(seqs, 32, 0, strand)
    eI, eD = oracle.matrix(off, codes, 0, 24, 0, 24)
    for mfma, sp, fs, lo in ((1, None, None, None), (0, 0, None, None), (0, 0, 0, None), (0, 0, 1, None),
                             (0, 0, 2, None), (0, 0, 4, None), (0, 0, None, 0), (0, None, None, 0)):
        if True:
            ctx.set_option("bitset_mfma", mfma)
            ctx.set_option("sparse", sp)
            ctx.set_option("fill_sort", fs)
            ctx.set_option("locus_order", lo)
            sets = gdist.KmerSets.from_sequences(seqs, 32, gdist.KmerType.DNA, strand, ctx)
            sets.build_bitsets(keep_singletons=True)
            I, D = sets.matrix(method=gdist.METHOD_BITSET)
            bad = np.argwhere(I != eI)
            print(f"strand {strand} mfma {mfma} sparse {sp} fill_sort {fs} locus {lo}: bitset_info {sets.bitset_info()} sparse_info "
                  f"{sets.sparse_info()} rare {sets.rare_info()} mismatches {len(bad)} "
                  f"{[(int(a), int(b), int(I[a, b]), int(eI[a, b])) for a, b in bad[:6]]}", flush=True)
ctx.close()
