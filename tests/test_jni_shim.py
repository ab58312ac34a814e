"""The JNI shim (jni/gdist_jni.c) cannot be compiled here (no JDK, no jni.h);
these checks hold it to the C-ABI it binds instead: every gdist_* call names a
function include/gdist.h declares, with that function's number of arguments;
every native of jni/GpuKmerSets.java has its JNIEXPORT and vice versa; and no
JVM array is pinned across a library call (GetPrimitiveArrayCritical)."""
import os
import re

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
