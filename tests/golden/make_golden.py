"""Generates tests/golden/kmer_golden.json from the pure-Python string-set
restatement (oracle/pyref.py) and refuses to write unless the C oracle
(oracle/gdist_oracle.c) agrees bit for bit.

PARITY UNPINNED: no reference output exists for this path (SURVEY.md §8c:
the kmer classes are in the un-vendored org.theseed:sequence module and no
JVM is available), so these vectors pin the two independent restatements
to each other and, through the GPU tests, the HIP path to both.
Run: python tests/golden/make_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402
import pyref  # noqa: E402

DNA, PROT = 0, 1


def rand_seqs(rng, alpha, n, lmin, lmax, base=None, mut=0.1):
    out = []
    for _ in range(n):
        if base is not None and rng.random() < 0.7:
            s = list(base[: rng.randint(lmin, min(lmax, len(base)))])
            for i in range(len(s)):
                if rng.random() < mut:
                    s[i] = rng.choice(alpha)
            out.append("".join(s))
        else:
            out.append("".join(rng.choice(alpha) for _ in range(rng.randint(lmin, lmax))))
    return out


def case(name, kind, k, flags, seqs, width=16):
    sets = [pyref.kmer_set(s, k, kind, flags) for s in seqs]
    n = len(sets)
    I = [[len(sets[i] & sets[j]) for j in range(n)] for i in range(n)]
    D = [[pyref.java_double_str(pyref.set_distance(sets[i], sets[j])) for j in range(n)] for i in range(n)]
    codes = [sorted(pyref.encode(x, kind, flags) for x in s) for s in sets]
    sk = [pyref.sketch(s, width) for s in sets]
    skD = [[pyref.java_double_str(pyref.sketch_distance(sk[i], sk[j], width)[0]) for j in range(n)] for i in range(n)]
    skJ = [[pyref.java_double_str(pyref.sketch_distance(sk[i], sk[j], width, pyref.SKETCH_JACCARD)[0])
            for j in range(n)] for i in range(n)]
    # the C oracle must agree before anything is written
    for s, c in zip(seqs, codes):
        got = [int(x) for x in oracle.kmer_codes(s.encode("latin-1"), k, kind, flags)]
        assert got == c, (name, s)
    for i in range(n):
        ci = np.array(codes[i], dtype=np.uint64)
        got_sk = [int(x) for x in oracle.sketch(ci, k, kind, width, flags)]
        assert got_sk == sk[i], (name, i)
        for j in range(n):
            cj = np.array(codes[j], dtype=np.uint64)
            Ii = oracle.intersect(ci, cj)
            assert Ii == I[i][j]
            assert oracle.java_dtoa(oracle.distance(Ii, len(ci), len(cj))) == D[i][j]
            assert oracle.java_dtoa(oracle.sketch_distance(np.array(sk[i], np.int32), np.array(sk[j], np.int32),
                                                           width)[0]) == skD[i][j]
    return {"name": name, "kind": kind, "k": k, "flags": flags, "seqs": seqs, "sizes": [len(s) for s in sets],
            "codes": [[str(x) for x in c] for c in codes], "I": I, "D": D, "width": width,
            "sketch": sk, "sketch_D": skD, "sketch_D_jaccard": skJ}


def main():
    rng = random.Random(20250725)
    cases = []
    anc = "".join(rng.choice("ACGT") for _ in range(400))
    cases.append(case("dna_both_k9", DNA, 9, 0x0, rand_seqs(rng, "ACGT", 10, 0, 300, anc, 0.03)))
    cases.append(case("dna_mixed_case_ambig_k7", DNA, 7, 0x0,
                      rand_seqs(rng, "ACGTacgtNnRx", 8, 0, 120, anc.lower(), 0.05) + ["", "ACG", "acgtacgtAAAAAAAAAA"]))
    cases.append(case("dna_fwd_k5", DNA, 5, 0x1, rand_seqs(rng, "ACGT", 8, 0, 150, anc, 0.05)))
    cases.append(case("dna_canon_k11", DNA, 11, 0x2, rand_seqs(rng, "ACGT", 8, 0, 200, anc, 0.02)))
    cases.append(case("dna_keep_k6", DNA, 6, 0x8, rand_seqs(rng, "ACGTNRY", 8, 0, 100, anc, 0.1)))
    cases.append(case("dna_k21_contigs", DNA, 21, 0x0,
                      ["\0".join(rand_seqs(rng, "ACGT", 3, 20, 120, anc, 0.01)) for _ in range(6)]))
    panc = "".join(rng.choice("ACDEFGHIKLMNPQRSTVWY") for _ in range(300))
    cases.append(case("prot_k8", PROT, 8, 0x0, rand_seqs(rng, "ACDEFGHIKLMNPQRSTVWY", 10, 0, 250, panc, 0.05)))
    cases.append(case("prot_k3_case_x", PROT, 3, 0x0, rand_seqs(rng, "ACDEFGacdefgX*", 8, 0, 80, panc, 0.2)))
    cases.append(case("prot_k3_nofold", PROT, 3, 0x10, rand_seqs(rng, "ACDacdX*", 6, 0, 60)))
    cases.append(case("prot_k10_5bit", PROT, 10, 0x0, rand_seqs(rng, "ACDEFGHIKLMNPQRSTVWYX*", 8, 0, 150, panc, 0.05)))
    cases.append(case("prot_skip_k4", PROT, 4, 0x4, rand_seqs(rng, "ACDEFGHIKX*", 8, 0, 80, panc, 0.1)))
    cases.append(case("known_answers", DNA, 3, 0x1, ["ACGTT", "CGTTA", "ACGTT", "GGGGG", "AC", "AAAAAA"]))
    path = os.path.join(HERE, "kmer_golden.json")
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (oracle/pyref.py, cross-checked by oracle/gdist_oracle.c)",
                   "parity": "unpinned (no reference vectors exist; SURVEY.md 8c)", "cases": cases}, f)
    print("wrote", path, os.path.getsize(path), "bytes,", len(cases), "cases")


if __name__ == "__main__":
    main()
