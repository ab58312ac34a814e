"""CPU: the C oracle against the golden vectors, the independent Python
restatement and hand-derived known answers (parity unpinned: SURVEY §8c)."""
import json
import math
import os
import random

import numpy as np
import pytest

import oracle
import pyref
from gdist.javafmt import java_double

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kmer_golden.json")


def load_cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", load_cases(), ids=lambda c: c["name"])
def test_oracle_matches_golden(case):
    kind, k, flags = case["kind"], case["k"], case["flags"]
    codes = [oracle.kmer_codes(s.encode("latin-1"), k, kind, flags) for s in case["seqs"]]
    assert [len(c) for c in codes] == case["sizes"]
    for c, exp in zip(codes, case["codes"]):
        assert [str(int(x)) for x in c] == exp
    off = np.zeros(len(codes) + 1, np.int64)
    off[1:] = np.cumsum([len(c) for c in codes])
    flat = np.concatenate(codes) if codes else np.zeros(0, np.uint64)
    n = len(codes)
    I, D = oracle.matrix(off, flat, 0, n, 0, n)
    assert I.tolist() == case["I"]
    assert [[oracle.java_dtoa(x) for x in row] for row in D] == case["D"]
    w = case["width"]
    sk = [oracle.sketch(c, k, kind, w, flags) for c in codes]
    assert [s.tolist() for s in sk] == case["sketch"]
    for i in range(n):
        for j in range(n):
            d, _ = oracle.sketch_distance(sk[i], sk[j], w)
            assert oracle.java_dtoa(d) == case["sketch_D"][i][j]
            dj, _ = oracle.sketch_distance(sk[i], sk[j], w, pyref.SKETCH_JACCARD)
            assert oracle.java_dtoa(dj) == case["sketch_D_jaccard"][i][j]


def test_known_answers():
    # identical sets -> 0.0, disjoint -> 1.0 (GroupTypeSpec.java:84 treats 1.0 as "nothing shared")
    a = oracle.kmer_codes(b"ACGTT", 3, 0, pyref.STRAND_FWD)
    b = oracle.kmer_codes(b"CGTTA", 3, 0, pyref.STRAND_FWD)
    assert len(a) == 3 and len(b) == 3
    assert oracle.intersect(a, a) == 3 and oracle.java_dtoa(oracle.distance(3, 3, 3)) == "0.0"
    # worked example: {ACG,CGT,GTT} vs {CGT,GTT,TTA}: I=2, union 4 -> 0.5
    assert oracle.intersect(a, b) == 2
    assert oracle.java_dtoa(oracle.distance(2, 3, 3)) == "0.5"
    g = oracle.kmer_codes(b"GGGGG", 3, 0, pyref.STRAND_FWD)
    assert oracle.intersect(a, g) == 0 and oracle.java_dtoa(oracle.distance(0, 3, 1)) == "1.0"
    # repeated kmers collapse; shorter than k -> empty; empty vs empty -> 1.0 (NaN mode available)
    assert len(oracle.kmer_codes(b"AAAAAA", 3, 0, pyref.STRAND_FWD)) == 1
    assert len(oracle.kmer_codes(b"AC", 3, 0, 0)) == 0
    assert oracle.distance(0, 0, 0) == 1.0
    assert math.isnan(oracle.distance(0, 0, 0, pyref.EMPTY_NAN))
    # both strands: ACGT is its own reverse complement -> {AC, CG, GT}
    assert len(oracle.kmer_codes(b"ACGT", 2, 0, pyref.STRAND_BOTH)) == 3
    # case folding and ambiguity skip (DNA default): acgNt -> only 'ACG' (k=3)
    assert [int(x) for x in oracle.kmer_codes(b"acgNt", 3, 0, pyref.STRAND_FWD)] == [pyref.encode("ACG")]
    # 1 - 1/3
    assert oracle.java_dtoa(oracle.distance(1, 2, 2)) == "0.6666666666666667"


@pytest.mark.parametrize("v,s", [(0.5, "0.5"), (1.0, "1.0"), (0.0, "0.0"), (9.5e-4, "9.5E-4"), (1e-3, "0.001"),
                                 (1e7, "1.0E7"), (1e-5, "1.0E-5"), (4.9e-324, "4.9E-324"), (1e23, "1.0E23"),
                                 (123456.789, "123456.789"), (float("nan"), "NaN"), (-0.0, "-0.0"),
                                 (float("inf"), "Infinity"), (2.0 / 3.0, "0.6666666666666666")])
def test_java_double_to_string(v, s):
    assert oracle.java_dtoa(v) == s
    assert pyref.java_double_str(v) == s
    assert java_double(v) == s


def test_java_format_random_agreement():
    rng = random.Random(7)
    for _ in range(20000):
        i = rng.randint(0, 10 ** 6)
        na, nb = rng.randint(i, 10 ** 6), rng.randint(i, 10 ** 6)
        d = pyref.distance(i, na, nb)
        assert oracle.java_dtoa(d) == pyref.java_double_str(d) == java_double(d)
        x = rng.random() * 10 ** rng.randint(-12, 12)
        assert oracle.java_dtoa(x) == pyref.java_double_str(x) == java_double(x)


def test_oracle_vs_pyref_random():
    rng = random.Random(11)
    for _ in range(1500):
        kind = rng.choice([0, 1])
        if kind == 0:
            alpha = rng.choice(["ACGT", "acgtACGT", "ACGTN", "ACGTNRYacgt", "ACGT\0"])
            flags = rng.choice([0, 1, 2]) | rng.choice([0, 4, 8])
            k = rng.randint(1, 21)
        else:
            alpha = rng.choice(["ACDEFGHIKLMNPQRSTVWY", "ACDEFGHIKLMNPQRSTVWYX*", "acdefgACD", "AC1", "ACD\0"])
            flags = rng.choice([0, 4, 8]) | rng.choice([0, 0x10])
            k = rng.randint(1, 12)
        s = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 50)))
        try:
            c = [int(x) for x in oracle.kmer_codes(s.encode("latin-1"), k, kind, flags)]
        except ValueError:
            c = None
        try:
            e = sorted(pyref.encode(x, kind, flags) for x in pyref.kmer_set(s, k, kind, flags))
        except ValueError:
            e = None
        assert c == e


def test_murmur3_and_sketch_vs_pyref():
    rng = random.Random(3)
    for _ in range(300):
        b = bytes(rng.randrange(256) for _ in range(rng.randint(0, 40)))
        assert oracle.murmur3(b) == pyref.murmur3_32(b)
    seq = "".join(rng.choice("ACGT") for _ in range(500))
    codes = oracle.kmer_codes(seq.encode(), 11, 0, 0)
    for w in (1, 10, 100, 5000):
        assert oracle.sketch(codes, 11, 0, w).tolist() == pyref.sketch(pyref.kmer_set(seq, 11), w)


def test_faithful_path_matches_oracle():
    """The Java-faithful HashSet<String> baseline computes the same distances."""
    rng = random.Random(5)
    anc = "".join(rng.choice("ACGT") for _ in range(600))
    seqs = ["".join(c if rng.random() > 0.02 else rng.choice("ACGT") for c in anc) for _ in range(25)]
    pairs, D = oracle.faithful_fasta_dist([s.encode() for s in seqs], 11, 0, 0, batch=20)
    assert pairs == 25 * 24 // 2
    off, codes = oracle.pack([s.encode() for s in seqs], 11)
    _, Dm = oracle.matrix(off, codes, 0, 25, 0, 25, flags=0x100)
    iu = np.triu_indices(25, 1)
    assert np.array_equal(D[iu], Dm[iu])


def test_java_format_f_half_up_on_shortest_digits():
    from gdist.javafmt import java_format_f
    assert java_format_f(0.03125, 8, 4) == "  0.0313"      # Python "%8.4f" gives 0.0312
    assert java_format_f(1.0005, 8, 3) == "   1.001"       # shortest digits, not the exact binary value
    assert java_format_f(0.0, 8, 4) == "  0.0000"
    assert java_format_f(-1e-05, 8, 4) == " -0.0000"
    assert java_format_f(float("nan"), 8, 4) == "     NaN"


def test_width_processor_validation_and_sizes():
    import pytest
    from gdist import processors as P
    assert P.sketch_sizes(50, 100, 25) == [50, 75, 100]
    assert P.sketch_sizes(50, 60, 20) == [50]
    for kw, msg in ((dict(min_size=20, max_size=10), "Minimum"), (dict(step=0), "Step"),
                    (dict(max_group=5), "group size"), (dict(target_error=0.2), "Target")):
        args = dict(min_size=10, max_size=20)
        args.update(kw)
        with pytest.raises(P.ParseFailureException, match=msg):
            P.width_processor([], out=None, **args)


def test_java_string_hash_and_hashmap_order():
    from gdist.processors import java_hashmap_order, java_string_hash
    assert java_string_hash("hello") == 99162322
    assert java_string_hash("") == 0
    assert java_string_hash("Aa") == java_string_hash("BB") == 2112
    assert java_string_hash("polygenelubricants") == -2147483648        # a known Integer.MIN_VALUE hash
    # 3 keys: table of 16, buckets (h ^ h>>>16) & 15, insertion order within a bucket
    keys = ["b", "a", "Aa", "BB"]
    assert java_hashmap_order(keys) == sorted(range(4), key=lambda i: ((java_string_hash(keys[i]) & 0xFFFFFFFF ^
                                                                         (java_string_hash(keys[i]) & 0xFFFFFFFF) >> 16) & 15, i))
    assert java_hashmap_order(["Aa", "BB"]) == [0, 1] and java_hashmap_order(["BB", "Aa"]) == [0, 1]


def test_hashmap_order_initial_capacity():
    """repMap is `new HashMap<>(500)` (DistanceRepsProcessor.java:175): a
    512-bucket table from the first put, grown only past 384 keys. Hand
    computed: String.hashCode of a one-char key is its char (a=97, b=98,
    q=113), the spread h ^ h>>>16 leaves it, so with 16 buckets a and q share
    bucket 1 (b is 2) and with 512 buckets they are 97, 98, 113."""
    from gdist.processors import DISTREPS_REPMAP_CAPACITY, java_hashmap_order, java_table_size_for
    assert java_table_size_for(500) == 512 and java_table_size_for(100) == 128 and java_table_size_for(16) == 16
    keys = ["q", "b", "a"]
    assert java_hashmap_order(keys) == [0, 2, 1]                                    # q(1) a(1) b(2)
    assert java_hashmap_order(keys, DISTREPS_REPMAP_CAPACITY) == [2, 1, 0]          # a(97) b(98) q(113)
    # 20 keys where bucket mod 16 and bucket mod 512 give different orders
    many = [chr(ord("A") + i) + chr(ord("a") + (7 * i) % 26) for i in range(20)]
    o16, o512 = java_hashmap_order(many), java_hashmap_order(many, 500)
    assert o16 != o512 and sorted(o16) == sorted(o512) == list(range(20))
    # two-char keys: hashCode = 31*c0 + c1 < 512*16, spread is the identity below 2^16
    assert o512 == sorted(range(20), key=lambda i: ((31 * ord(many[i][0]) + ord(many[i][1])) & 511, i))
    # growth: 384 keys stay in 512 buckets, the 385th put resizes to 1024
    k385 = ["k%d" % i for i in range(385)]
    def h(s):
        x = 0
        for ch in s:
            x = (31 * x + ord(ch)) & 0xFFFFFFFF
        return x ^ (x >> 16)
    assert java_hashmap_order(k385[:384], 500) == sorted(range(384), key=lambda i: (h(k385[i]) & 511, i))
    assert java_hashmap_order(k385, 500) == sorted(range(385), key=lambda i: (h(k385[i]) & 1023, i))


def test_lsh_oracle_known_answer():
    """oracle.lsh_closest (the restated bucket search): with one bucket per
    stage every indexed sketch is a candidate; distances are the Mash
    bottom-s distances, nearest first, ties by index, capped at n."""
    s = [np.array([1, 5, 9, 12], np.int32), np.array([1, 5, 9, 13], np.int32), np.array([100, 200], np.int32)]
    assert oracle.lsh_closest(s, [s[0]], 8, 3, 1, 1, 5, 1.0) == [[(0, 0.0), (1, 0.4), (2, 1.0)]]
    assert oracle.lsh_closest(s, [s[0]], 8, 3, 1, 1, 2, 1.0) == [[(0, 0.0), (1, 0.4)]]
    assert oracle.lsh_closest(s, [s[0]], 8, 3, 1, 1, 5, 0.3) == [[(0, 0.0)]]
    b = oracle.lsh_buckets(s[0], 4, 1000, 7)
    assert len(b) == 4 and all(0 <= x < 1000 for x in b) and b == oracle.lsh_buckets(list(s[0]), 4, 1000, 7)
