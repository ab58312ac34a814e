"""The JNI shim (jni/gdist_jni.c). No JDK exists in this image, so:
* static checks hold it to the C-ABI it binds: every gdist_* call names a
  function include/gdist.h declares, with that function's number of
  arguments; every native of jni/GpuKmerSets.java has its JNIEXPORT and vice
  versa; no JVM array is pinned across a library call;
* it is COMPILED with gcc -Wall -Wextra -Werror against a test-only JNI
  stand-in (tests/jni_harness: the JNI specification's types and signatures
  of the functions it uses, and an in-process fake JVM) and its natives are
  called through ctypes as a JVM would call them: argument validation and the
  status -> exception mapping on the CPU, and (-m gpu) pack / matrix / row
  queries / greedy reps / sketches on the device against the oracle.
"""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(*p):
    with open(os.path.join(ROOT, *p)) as f:
        return f.read()


def _split_args(s):
    """Top-level comma split of an argument list (parentheses aware)."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def _calls(src, prefix):
    """(name, argument count) of every call name(...) with the prefix."""
    for m in re.finditer(r"\b(" + prefix + r"\w+)\s*\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        yield m.group(1), len(_split_args(src[m.end():i - 1]))


def _header_arity():
    h = re.sub(r"/\*.*?\*/", "", _read("include", "gdist.h"), flags=re.S)
    decl = {}
    for m in re.finditer(r"\b(?:int|const char\*)\s+(gdist_\w+)\s*\(([^;]*?)\)\s*;", h):
        args = m.group(2).strip()
        decl[m.group(1)] = 0 if args in ("", "void") else len(_split_args(args))
    return decl


def test_shim_calls_match_header():
    src = re.sub(r"/\*.*?\*/", "", _read("jni", "gdist_jni.c"), flags=re.S)
    decl = _header_arity()
    seen = set()
    for name, n in _calls(src, "gdist_"):
        assert name in decl, f"{name} is not declared in include/gdist.h"
        assert n == decl[name], f"{name}: {n} arguments, gdist.h declares {decl[name]}"
        seen.add(name)
    for need in ("gdist_sets_pack", "gdist_intersect_matrix", "gdist_row_query", "gdist_greedy_reps",
                 "gdist_sketch_build", "gdist_sketch_matrix", "gdist_last_error"):
        assert need in seen, need


def test_natives_pair_up_and_no_critical_sections():
    c = _read("jni", "gdist_jni.c")
    java = _read("jni", "GpuKmerSets.java")
    exported = set(re.findall(r"JNIEXPORT\s+\w+\s+JNICALL\s+JFN\((\w+)\)", c))
    natives = set(re.findall(r"static native \w+(?:\[\])?\s+(\w+)\s*\(", java))
    assert exported and exported == natives, (exported ^ natives)
    assert "GetPrimitiveArrayCritical" not in re.sub(r"/\*.*?\*/", "", c, flags=re.S)
    assert "package org.theseed.genome.distance.gpu;" in java
    assert "#define JFN(name) Java_org_theseed_genome_distance_gpu_GpuKmerSets_##name" in c


@pytest.fixture(scope="module")
def jvm(tmp_path_factory):
    """The shim + fake JVM: the in-tree build of __graft_entry__.build() when
    it is newer than its sources, else compiled here (gcc, about a second)."""
    from jni_harness import harness
    return harness.FakeJVM(harness.current() or
                           harness.build(str(tmp_path_factory.mktemp("jni") / "libgdist_jni_test.so")))


def test_shim_compiles_and_maps_errors(jvm):
    """Compiled with -Werror against the JNI signatures; every failure path
    leaves exactly the exception SURVEY §8b maps its status to, and the shim
    returns without touching a Java array after an exception."""
    from jni_harness.harness import LONG, DOUBLE, INT
    import ctypes as C
    # a null collection: EINVAL -> IllegalArgumentException with gdist_last_error()
    out = jvm.zeros(LONG, 4)
    jvm.call("nSizes", None, 0, C.c_void_p(out))
    cls, msg = jvm.exception()
    assert cls == "java/lang/IllegalArgumentException" and msg
    assert jvm.call("nSize", C.c_int64, 0) == 0
    assert jvm.exception()[0] == "java/lang/IllegalArgumentException"
    # an output array shorter than (r1 - r0) * ld is refused before any call
    d = jvm.zeros(DOUBLE, 5)
    jvm.call_i("nMatrix", None, [C.c_int64] * 6 + [C.c_int32, C.c_int32, C.c_void_p, C.c_int32],
               0, 0, 0, 3, 0, 3, 0, 0x100, d, 3)
    assert jvm.exception() == ("java/lang/IllegalArgumentException", "output array smaller than (r1 - r0) * ld")
    # greedy reps on a null collection: refused before any array is read
    ir = jvm.zeros(INT, 3)
    jvm.call("nGreedyReps", C.c_int64, 0, 0, 0.5, C.c_void_p(None), C.c_void_p(ir), C.c_void_p(None),
             C.c_void_p(None))
    assert jvm.exception()[0] == "java/lang/IllegalArgumentException"
    # row queries: the cols copy, then the library's EINVAL for the null handle
    cols = jvm.array(LONG, [0, 1])
    assert jvm.call("nAnyLe", C.c_uint8, 0, 0, 0, C.c_void_p(cols), 0.5) == 0
    assert jvm.exception()[0] == "java/lang/IllegalArgumentException"
    short = jvm.zeros(DOUBLE, 1)
    jvm.call("nRow", None, 0, 0, 0, C.c_void_p(cols), C.c_void_p(short))
    assert jvm.exception() == ("java/lang/IllegalArgumentException", "out shorter than cols")
    # options by name (a null context: EINVAL)
    jvm.call("nSetOption", None, 0, C.c_void_p(jvm.string("sparse")), 1)
    assert jvm.exception()[0] == "java/lang/IllegalArgumentException"
    assert jvm.lib.fj_local_refs() == 0


@pytest.mark.gpu
def test_shim_on_device_vs_oracle(jvm):
    """The natives a Java host calls, end to end on the GPU: nCtxCreate, nPack
    (KmerType.createKmers for a batch), nSizes, nMatrix (the fastaDist row
    blocks, upper triangle), nRow / nAnyLe / nArgmin (DistanceRepsProcessor's
    row queries), nGreedyReps (with the one-element-per-set contract
    enforced), nSketch + nSketchMatrix, nFree, nCtxDestroy — against the oracle."""
    import ctypes as C
    import oracle
    from gdist import synth
    from jni_harness.harness import LONG, DOUBLE, INT
    n = 40
    seqs = [bytes(r) for r in synth.genomes(n, 4000, 0.02, 31)]
    off, codes = oracle.pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, n, 0, n, flags=0x100)
    ctx = jvm.call_i("nCtxCreate", C.c_int64, [C.c_int32], 0)
    assert jvm.exception() is None and ctx
    sets = jvm.call_i("nPack", C.c_int64, [C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_void_p],
                      ctx, 0, 21, 0, jvm.byte_arrays(seqs))
    assert jvm.exception() is None and sets
    assert jvm.lib.fj_local_refs() == 0                     # every element reference deleted
    assert jvm.call("nSize", C.c_int64, sets) == n
    sz = jvm.zeros(LONG, n)
    jvm.call("nSizes", None, sets, C.c_void_p(sz))
    assert jvm.exception() is None and jvm.read(sz, LONG, n) == np.diff(off).tolist()
    jvm.call("nSizes", None, sets, C.c_void_p(jvm.zeros(LONG, n - 1)))
    assert jvm.exception() == ("java/lang/IllegalArgumentException", "out shorter than the number of sets")
    d = jvm.array(DOUBLE, [7.5] * (n * n))
    jvm.call_i("nMatrix", None, [C.c_int64] * 6 + [C.c_int32, C.c_int32, C.c_void_p, C.c_int32],
               ctx, sets, 0, n, 0, n, 0, 0x100, d, n)
    assert jvm.exception() is None
    D = np.array(jvm.read(d, DOUBLE, n * n)).reshape(n, n)
    iu = np.triu_indices(n, 1)
    assert np.array_equal(D[iu].view(np.uint64), eD[iu].view(np.uint64))
    assert np.all(D[np.tril_indices(n)] == 7.5)              # below the diagonal: the caller's values
    cols = [3, 0, 39, 17]
    row = jvm.zeros(DOUBLE, 4)
    jvm.call("nRow", None, ctx, sets, 5, C.c_void_p(jvm.array(LONG, cols)), C.c_void_p(row))
    _, eR = oracle.matrix(off, codes, 5, 6, 0, n)
    assert jvm.exception() is None and np.array_equal(np.array(jvm.read(row, DOUBLE, 4)).view(np.uint64),
                                                      eR[0, cols].view(np.uint64))
    t = float(np.sort(eR[0, cols])[1])
    assert jvm.call("nAnyLe", C.c_uint8, ctx, sets, 5, C.c_void_p(jvm.array(LONG, cols)), t) == 1
    best = jvm.zeros(DOUBLE, 1)
    k = jvm.call("nArgmin", C.c_int32, ctx, sets, 5, C.c_void_p(jvm.array(LONG, cols)), C.c_void_p(best))
    assert jvm.exception() is None and eR[0, cols[k]] == eR[0, cols].min() == jvm.read(best, DOUBLE, 1)[0]
    # greedy reps: every array one element per set (a short one is refused, no write)
    ir, ro, rd = jvm.zeros(INT, n), jvm.zeros(LONG, n), jvm.zeros(DOUBLE, n)
    jvm.call("nGreedyReps", C.c_int64, ctx, sets, 0.5, C.c_void_p(None), C.c_void_p(ir), C.c_void_p(jvm.zeros(LONG, 3)),
             C.c_void_p(rd))
    assert jvm.exception() == ("java/lang/IllegalArgumentException", "repOf shorter than the number of sets")
    nreps = jvm.call("nGreedyReps", C.c_int64, ctx, sets, 0.5, C.c_void_p(None), C.c_void_p(ir), C.c_void_p(ro),
                     C.c_void_p(rd))
    assert jvm.exception() is None
    is_rep = jvm.read(ir, INT, n)
    assert nreps == sum(is_rep) and is_rep[0] == 1
    _, full = oracle.matrix(off, codes, 0, n, 0, n)
    reps = []
    for i in range(n):                                      # DistanceRepsProcessor.java:185-201
        if not any(full[i, r] <= 0.5 for r in reps):
            reps.append(i)
    assert [i for i in range(n) if is_rep[i]] == reps
    # sketches: hashSet(64) of every set and Sketch.distance over the triangle
    sk = jvm.call_i("nSketch", C.c_int64, [C.c_int64, C.c_int64, C.c_int32], ctx, sets, 64)
    assert jvm.exception() is None and sk
    sd = jvm.zeros(DOUBLE, n * n)
    jvm.call_i("nSketchMatrix", None, [C.c_int64] * 6 + [C.c_int32, C.c_void_p, C.c_int32],
               ctx, sk, 0, n, 0, n, 0x100, sd, n)
    SD = np.array(jvm.read(sd, DOUBLE, n * n)).reshape(n, n)
    ref = [oracle.sketch(codes[off[i]:off[i + 1]], 21, 0, 64) for i in range(n)]
    for i, j in zip(*iu):
        assert SD[i, j] == oracle.sketch_distance(ref[i], ref[j], 64)[0]
    for h in (sk, sets):
        jvm.call("nFree", None, h)
        assert jvm.exception() is None
    jvm.call("nCtxDestroy", None, ctx)
    assert jvm.exception() is None


class _KmerMethodMirror:
    """jni/GpuKmerMethod.java + GpuMeasurer.java, statement for statement, over
    the shim's natives: setOf packs a genome the first time its id is seen
    (nPack for the first, nAppend after); getMeasurer restarts a full cache
    (parameter cache=N) and holds id1's set; a measurer's first getDistance
    takes id1's row against every cached genome (one nMatrix of one row) and
    answers later pairs from it, asking again only for a genome appended
    after the row was taken."""

    def __init__(self, jvm, ctx, k, cache_limit=4096):
        self.jvm, self.ctx, self.k = jvm, ctx, k
        self.cache = 0
        self.set_index = {}
        self.packs = 0
        self.cache_limit = cache_limit
        self.generation = 0
        self.device_calls = 0

    def set_of(self, gid, seq):
        import ctypes as C
        i = self.set_index.get(gid)
        if i is None:
            arr = self.jvm.byte_arrays([seq])
            if self.cache == 0:
                self.cache = self.jvm.call_i("nPack", C.c_int64, [C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                                                  C.c_void_p], self.ctx, 0, self.k, 0, arr)
                i = 0
            else:
                i = self.jvm.call("nAppend", C.c_int64, self.ctx, self.cache, C.c_void_p(arr))
            assert self.jvm.exception() is None
            self.packs += 1
            self.set_index[gid] = i
        return i

    def row(self, i):
        """GpuKmerMethod.row: distances(i, i + 1, 0, n, false, d, n) -> nMatrix, METHOD_AUTO"""
        import ctypes as C
        from jni_harness.harness import DOUBLE
        n = self.jvm.call("nSize", C.c_int64, self.cache)
        d = self.jvm.zeros(DOUBLE, max(n, 1))
        self.jvm.call_i("nMatrix", None, [C.c_int64] * 6 + [C.c_int32, C.c_int32, C.c_void_p, C.c_int32],
                        self.ctx, self.cache, i, i + 1, 0, n, 0, 0, d, n)
        assert self.jvm.exception() is None
        self.device_calls += 1
        return self.jvm.read(d, DOUBLE, n)

    def get_measurer(self, gid, seq):
        if self.cache != 0 and len(self.set_index) >= self.cache_limit:
            self.jvm.call("nFree", None, self.cache)
            self.cache = 0
            self.set_index.clear()
            self.generation += 1
        return _MeasurerMirror(self, gid, seq)


class _MeasurerMirror:
    def __init__(self, method, gid, seq):
        self.method, self.gid, self.seq = method, gid, seq
        self.set1 = method.set_of(gid, seq)
        self.gen = method.generation
        self.row = None

    def distance_to(self, gid2, seq2):
        if self.gen != self.method.generation:
            self.set1 = self.method.set_of(self.gid, self.seq)
            self.gen = self.method.generation
            self.row = None
        j = self.method.set_of(gid2, seq2)
        if self.row is None or j >= len(self.row):
            self.row = self.method.row(self.set1)
        return self.row[j]


@pytest.mark.gpu
@pytest.mark.parametrize("cache_limit", [4096, 8])
def test_java_measurer_packs_each_genome_once(jvm, cache_limit):
    """the `methods` drop-in (GpuKmerMethod /
    GpuMeasurer) driven as MethodTableProcessor drives it (pairs grouped by
    id1, GenomePairList.prepare :240; getMeasurer per group :261-265;
    getDistance per pair :275): every genome is packed once (nPack / nAppend)
    while the cache holds it, a group whose second genomes are all cached
    costs ONE device call (its id1 row), and every distance equals the
    oracle's. With a small cache bound the cache restarts between
    groups and the distances stay exact."""
    import ctypes as C
    import random
    import oracle
    from gdist import synth
    n = 24
    seqs = [bytes(r) for r in synth.genomes(n, 6000, 0.03, 37)]
    off, codes = oracle.pack(seqs, 21, 0, 0)
    _, eD = oracle.matrix(off, codes, 0, n, 0, n)
    rng = random.Random(5)
    pairs = sorted({(rng.randrange(n), rng.randrange(n)) for _ in range(120)})   # grouped by id1
    groups = len({a for a, _ in pairs})
    ctx = jvm.call_i("nCtxCreate", C.c_int64, [C.c_int32], 0)
    m = _KmerMethodMirror(jvm, ctx, 21, cache_limit)
    for rnd in range(2):                                # the second pass: every genome cached
        calls0, packs0 = m.device_calls, m.packs
        id1, meas = None, None
        for a, b in pairs:
            if a != id1:                                # a new first genome: getMeasurer
                id1, meas = a, m.get_measurer(f"g{a}", seqs[a])
            d = meas.distance_to(f"g{b}", seqs[b])
            assert np.float64(d).view(np.uint64) == eD[a, b].view(np.uint64), (a, b, d, eD[a, b])
        if cache_limit >= n:
            if rnd == 0:
                assert m.packs == len({x for p in pairs for x in p})          # once per genome
            else:
                assert m.packs == packs0 and m.device_calls - calls0 == groups, (m.device_calls - calls0, groups)
        else:
            assert m.generation > 0
    if m.cache:
        assert jvm.call("nSize", C.c_int64, m.cache) == len(m.set_index)
        jvm.call("nFree", None, m.cache)
    jvm.call("nCtxDestroy", None, ctx)
    assert jvm.exception() is None


@pytest.mark.gpu
def test_java_genome_and_sketch_natives(jvm):
    """GpuGenomeProcessor's per-directory step (the base packed once,
    nConcat of the directory's sets and the base, row blocks of nMatrix) and
    GpuSketchProcessor's signatures (nSketch + nTotal + nSketchDownload)
    against the oracle."""
    import ctypes as C
    import oracle
    from gdist import synth
    from jni_harness.harness import LONG, DOUBLE, INT
    base = [bytes(r) for r in synth.genomes(9, 5000, 0.04, 38)]
    comp = [bytes(r) for r in synth.genomes(5, 5000, 0.04, 39)]
    ctx = jvm.call_i("nCtxCreate", C.c_int64, [C.c_int32], 0)
    pk = [C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]
    hb = jvm.call_i("nPack", C.c_int64, pk, ctx, 0, 21, 0, jvm.byte_arrays(base))
    hc = jvm.call_i("nPack", C.c_int64, pk, ctx, 0, 21, 0, jvm.byte_arrays(comp))
    both = jvm.call("nConcat", C.c_int64, hc, hb)
    assert jvm.exception() is None and jvm.call("nSize", C.c_int64, both) == 14
    m, nb = len(comp), len(base)
    off, codes = oracle.pack(comp + base, 21, 0, 0)
    _, eD = oracle.matrix(off, codes, 0, m, m, m + nb)
    rows = 2                                            # ROW_BLOCK_CELLS / nMain, scaled down
    for r0 in range(0, m, rows):
        r1 = min(m, r0 + rows)
        d = jvm.zeros(DOUBLE, rows * nb)
        jvm.call_i("nMatrix", None, [C.c_int64] * 6 + [C.c_int32, C.c_int32, C.c_void_p, C.c_int32],
                   ctx, both, r0, r1, m, m + nb, 0, 0, d, nb)
        assert jvm.exception() is None
        got = np.array(jvm.read(d, DOUBLE, (r1 - r0) * nb)).reshape(r1 - r0, nb)
        assert np.array_equal(got.view(np.uint64), eD[r0:r1].view(np.uint64))
    sk = jvm.call_i("nSketch", C.c_int64, [C.c_int64, C.c_int64, C.c_int32], ctx, hb, 100)
    total = jvm.call("nTotal", C.c_int64, sk)
    so, sv = jvm.zeros(LONG, nb + 1), jvm.zeros(INT, total)
    jvm.call("nSketchDownload", None, sk, C.c_void_p(so), C.c_void_p(sv))
    assert jvm.exception() is None
    o, v = jvm.read(so, LONG, nb + 1), jvm.read(sv, INT, total)
    bo, bc = oracle.pack(base, 21, 0, 0)
    for i in range(nb):
        assert v[o[i]:o[i + 1]] == list(oracle.sketch(bc[bo[i]:bo[i + 1]], 21, 0, 100)), i
    jvm.call("nSketchDownload", None, sk, C.c_void_p(jvm.zeros(LONG, nb)), C.c_void_p(sv))
    assert jvm.exception() == ("java/lang/IllegalArgumentException", "off shorter than the number of sets + 1")
    for h in (sk, both, hc, hb):
        jvm.call("nFree", None, h)
    jvm.call("nCtxDestroy", None, ctx)
    assert jvm.exception() is None


def test_sketch_upload_validates_arrays(jvm):
    """nSketchUpload refuses an empty offsets array and signatures shorter than
    off[nsets] before any library call (IllegalArgumentException)."""
    import ctypes as C
    from jni_harness.harness import LONG, INT
    up = [C.c_int64, C.c_int32, C.c_void_p, C.c_void_p]
    assert jvm.call_i("nSketchUpload", C.c_int64, up, 0, 10, jvm.zeros(LONG, 0), jvm.zeros(INT, 1)) == 0
    assert jvm.exception() == ("java/lang/IllegalArgumentException", "off needs nsets + 1 entries")
    assert jvm.call_i("nSketchUpload", C.c_int64, up, 0, 10, jvm.array(LONG, [0, 3, 5]), jvm.zeros(INT, 4)) == 0
    assert jvm.exception() == ("java/lang/IllegalArgumentException", "sigs shorter than off[nsets]")


@pytest.mark.gpu
def test_java_tuning_close_counts(jvm):
    """GpuTuningProcessor.closeCounts — the tune command's
    pair count (TuningProcessor.java:125-139: for each sketch the later
    sketches with distance < target) as one nSketchUpload of the Bucket's
    signatures and upper-triangle nSketchMatrix row blocks, counted per row —
    equals the reference loop restated over the oracle's Sketch.distance."""
    import ctypes as C
    import oracle
    from gdist import synth
    from jni_harness.harness import LONG, INT, DOUBLE
    n, width, target = 60, 120, 0.7
    prots = [bytes(r) for r in synth.genomes(n, 900, 0.25, 77, protein=True)]
    off, codes = oracle.pack(prots, 8, 1, 0)
    sigs = [oracle.sketch(codes[off[i]:off[i + 1]], 8, 1, width) for i in range(n)]
    sigs[7] = sigs[7][:40]                                # a dwarf
    # the restated reference loop
    expected = [sum(1 for j in range(i + 1, n) if oracle.sketch_distance(sigs[i], sigs[j], width)[0] < target)
                for i in range(n)]
    assert sum(expected) > 0 and sum(1 for e in expected if e == 0) > 0
    # closeCounts, statement for statement: width = the longest signature
    w = max(len(s) for s in sigs)
    so = np.zeros(n + 1, np.int64)
    so[1:] = np.cumsum([len(s) for s in sigs])
    ctx = jvm.call_i("nCtxCreate", C.c_int64, [C.c_int32], 0)
    sk = jvm.call_i("nSketchUpload", C.c_int64, [C.c_int64, C.c_int32, C.c_void_p, C.c_void_p], ctx, w,
                    jvm.array(LONG, so.tolist()), jvm.array(INT, [int(x) for s in sigs for x in s]))
    assert jvm.exception() is None and sk
    rows = 16                                             # ROW_BLOCK_CELLS / n, scaled down
    got = [0] * n
    d = jvm.zeros(DOUBLE, rows * n)
    for r0 in range(0, n, rows):
        r1 = min(n, r0 + rows)
        jvm.call_i("nSketchMatrix", None, [C.c_int64] * 6 + [C.c_int32, C.c_void_p, C.c_int32],
                   ctx, sk, r0, r1, 0, n, 0x100, d, n)
        assert jvm.exception() is None
        D = np.array(jvm.read(d, DOUBLE, rows * n)).reshape(rows, n)
        for i in range(r0, r1):
            got[i] = int(np.sum(D[i - r0, i + 1:] < target))
    assert got == expected
    jvm.call("nFree", None, sk)
    jvm.call("nCtxDestroy", None, ctx)
    assert jvm.exception() is None
