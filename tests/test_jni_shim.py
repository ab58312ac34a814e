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
