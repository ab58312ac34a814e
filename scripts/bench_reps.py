"""Greedy representatives: device (gdist_greedy_reps) vs the per-candidate
row-query loop, on synthetic collections; checks both pick the same sets."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome.distance_amd"))
import numpy as np
import gdist
from gdist import synth, processors as P

ctx = gdist.Context(0)
for (n, L, pmax, prot, k, t) in [(10000, 33333, 0.10, True, 8, 0.5), (1000, 2_000_000, 0.002, False, 21, 0.3),
                                 (20000, 100_000, 0.05, False, 21, 0.6)]:
    g = synth.genomes(n, L, pmax, 7, protein=prot)
    seqs = [bytes(r) for r in g]
    del g
    sets = gdist.KmerSets.from_sequences(seqs, k, gdist.KmerType.PROT if prot else gdist.KmerType.DNA, 0, ctx)
    del seqs
    t0 = time.perf_counter(); sets.prepare(); tp = time.perf_counter() - t0
    t0 = time.perf_counter(); is_rep = sets.greedy_reps(t); td = time.perf_counter() - t0
    t0 = time.perf_counter(); _, rep_of, rep_d = sets.greedy_reps(t, assign=True); ta = time.perf_counter() - t0
    nh = min(n, 2000)
    sub_keys = [str(i) for i in range(n)]
    t0 = time.perf_counter()
    reps = []
    for i in range(nh):
        if reps and sets.row_query(i, reps, gdist.QUERY_ANY_LE, t):
            continue
        reps.append(i)
    th = time.perf_counter() - t0
    same = reps == [int(i) for i in np.flatnonzero(is_rep[:nh])]
    print(f"n={n} L={L} {'prot' if prot else 'dna'} k={k} t={t}: reps={int(is_rep.sum())} prepare {tp:.2f}s "
          f"device pass1 {td:.2f}s pass1+2 {ta:.2f}s | host loop first {nh}: {th:.2f}s (same={same})", flush=True)
