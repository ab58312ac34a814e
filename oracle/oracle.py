"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product package. Parity unpinned
(see gdist_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        i64, u64p, i64p = C.c_int64, C.POINTER(C.c_uint64), C.POINTER(C.c_int64)
        L.or_kmer_codes.restype = i64
        L.or_kmer_codes.argtypes = [C.c_int, C.c_int, C.c_uint, C.c_char_p, i64, u64p]
        L.or_intersect.restype = i64
        L.or_intersect.argtypes = [u64p, i64, u64p, i64]
        L.or_distance.restype = C.c_double
        L.or_distance.argtypes = [i64, i64, i64, C.c_uint]
        L.or_java_dtoa.restype = C.c_int
        L.or_java_dtoa.argtypes = [C.c_double, C.c_char_p]
        L.or_murmur3_32.restype = C.c_uint32
        L.or_murmur3_32.argtypes = [C.c_char_p, C.c_int, C.c_uint32]
        L.or_sketch.restype = i64
        L.or_sketch.argtypes = [C.c_int, C.c_int, C.c_uint, u64p, i64, C.c_int, C.POINTER(C.c_int32)]
        L.or_sketch_distance.restype = C.c_double
        L.or_sketch_distance.argtypes = [C.POINTER(C.c_int32), i64, C.POINTER(C.c_int32), i64,
                                         C.c_int, C.c_uint, i64p]
        L.or_matrix.restype = None
        L.or_matrix.argtypes = [i64p, u64p, i64, i64, i64, i64, C.c_uint,
                                C.POINTER(C.c_int32), C.POINTER(C.c_double), i64, C.c_int]
        L.or_rows_vs_columns.restype = C.c_int
        L.or_rows_vs_columns.argtypes = [C.c_int, C.c_int, C.c_uint, C.c_void_p, i64p, i64, i64p, u64p, i64,
                                         i64p, i64p, C.c_int]
        L.or_faithful_fasta_dist.restype = i64
        L.or_faithful_fasta_dist.argtypes = [C.c_int, C.c_int, C.c_uint, C.c_char_p, i64p, i64,
                                             C.c_int, i64, C.POINTER(C.c_double), C.c_int]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def kmer_codes(seq: bytes, k: int, kind: int = 0, flags: int = 0) -> np.ndarray:
    out = np.empty(max(2 * len(seq), 1), dtype=np.uint64)
    n = lib().or_kmer_codes(kind, k, flags, seq, len(seq), _p(out, C.c_uint64))
    if n < 0:
        raise ValueError("unencodable sequence for this kmer spec")
    return out[:n].copy()


def rows_vs_columns(blob, coff: np.ndarray, row_codes: list[np.ndarray], k: int, kind: int = 0,
                    flags: int = 0, nthreads: int = 0):
    """(inter[len(row_codes), ncols], sizes[ncols]): each row set against the
    codes of every column blob[coff[j]:coff[j+1]], extracted on the fly (C,
    OpenMP over columns) — for a collection too large to pack on the host."""
    buf = np.frombuffer(blob, dtype=np.uint8) if not isinstance(blob, np.ndarray) else blob
    coff = np.ascontiguousarray(coff, np.int64)
    ncols = len(coff) - 1
    roff = np.zeros(len(row_codes) + 1, np.int64)
    roff[1:] = np.cumsum([len(r) for r in row_codes])
    rc = np.ascontiguousarray(np.concatenate(row_codes) if row_codes else np.zeros(1), np.uint64)
    inter = np.zeros((len(row_codes), ncols), np.int64)
    sizes = np.zeros(ncols, np.int64)
    rc_ = lib().or_rows_vs_columns(kind, k, flags, buf.ctypes.data, _p(coff, C.c_int64), ncols,
                                   _p(roff, C.c_int64), _p(rc, C.c_uint64), len(row_codes),
                                   _p(inter, C.c_int64), _p(sizes, C.c_int64), nthreads)
    if rc_ != 0:
        raise ValueError("unencodable sequence for this kmer spec")
    return inter, sizes


def pack(seqs: list[bytes], k: int, kind: int = 0, flags: int = 0):
    sets = [kmer_codes(s, k, kind, flags) for s in seqs]
    off = np.zeros(len(sets) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(s) for s in sets])
    codes = np.concatenate(sets) if sets else np.zeros(0, np.uint64)
    return off, codes.astype(np.uint64)


def intersect(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, np.uint64); b = np.ascontiguousarray(b, np.uint64)
    return int(lib().or_intersect(_p(a, C.c_uint64), len(a), _p(b, C.c_uint64), len(b)))


def distance(inter: int, na: int, nb: int, flags: int = 0) -> float:
    return float(lib().or_distance(inter, na, nb, flags))


def java_dtoa(d: float) -> str:
    buf = C.create_string_buffer(64)
    n = lib().or_java_dtoa(d, buf)
    return buf.raw[:n].decode()


def murmur3(data: bytes, seed: int = 0) -> int:
    h = lib().or_murmur3_32(data, len(data), seed)
    return h - (1 << 32) if h & 0x80000000 else h


def sketch(codes: np.ndarray, k: int, kind: int, width: int, flags: int = 0) -> np.ndarray:
    codes = np.ascontiguousarray(codes, np.uint64)
    out = np.empty(max(width, 1), dtype=np.int32)
    n = lib().or_sketch(kind, k, flags, _p(codes, C.c_uint64), len(codes), width, _p(out, C.c_int32))
    return out[:n].copy()


def sketch_distance(a: np.ndarray, b: np.ndarray, width: int, flags: int = 0):
    a = np.ascontiguousarray(a, np.int32); b = np.ascontiguousarray(b, np.int32)
    common = C.c_int64(0)
    d = lib().or_sketch_distance(_p(a, C.c_int32), len(a), _p(b, C.c_int32), len(b), width, flags,
                                 C.byref(common))
    return float(d), int(common.value)


def matrix(off: np.ndarray, codes: np.ndarray, r0: int, r1: int, c0: int, c1: int,
           flags: int = 0, nthreads: int = 0):
    off = np.ascontiguousarray(off, np.int64); codes = np.ascontiguousarray(codes, np.uint64)
    I = np.zeros((r1 - r0, c1 - c0), dtype=np.int32)
    D = np.zeros((r1 - r0, c1 - c0), dtype=np.float64)
    lib().or_matrix(_p(off, C.c_int64), _p(codes, C.c_uint64), r0, r1, c0, c1, flags,
                    _p(I, C.c_int32), _p(D, C.c_double), c1 - c0, nthreads)
    return I, D


def faithful_fasta_dist(seqs: list[bytes], k: int, kind: int = 0, flags: int = 0, batch: int = 20,
                        max_rows: int = 0, nthreads: int = 0):
    blob = b"".join(seqs)
    off = np.zeros(len(seqs) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    n = len(seqs)
    D = np.full((n, n), np.nan, dtype=np.float64)
    pairs = lib().or_faithful_fasta_dist(kind, k, flags, blob, _p(off, C.c_int64), n, batch, max_rows,
                                         _p(D, C.c_double), nthreads)
    return int(pairs), D


# ---------------------------------------------------------------- LSH (restated)
_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def lsh_salts(stages: int, seed: int) -> list[int]:
    """Stage salts of gdist_lsh_build (csrc/lsh.hip)."""
    return [_mix64((seed + 0x9E3779B97F4A7C15 * (t + 1)) & _M64) for t in range(stages)]


def lsh_buckets(sig, stages: int, buckets: int, seed: int) -> list[int]:
    """Stage t's bucket of one signature: min over x of mix(uint32(x) ^ salt_t) mod buckets."""
    out = []
    for salt in lsh_salts(stages, seed):
        m = min((_mix64((int(x) & 0xFFFFFFFF) ^ salt) for x in sig), default=_M64)
        out.append(m % buckets)
    return out


def lsh_closest(subject_sigs, query_sigs, width: int, stages: int, buckets: int, seed: int, n: int,
                max_dist: float):
    """getClosest(kmers, n, maxDist) (MashProcessor.java:150, FindProcessor.java:110)
    restated over the LSH of csrc/lsh.hip: candidates share a bucket with the
    query in some stage; sketch distance <= max_dist; nearest first, ties by
    index; at most n. Test infrastructure (parity unpinned: the reference's
    LSH classes are un-vendored)."""
    index = {}
    for i, s in enumerate(subject_sigs):
        for t, b in enumerate(lsh_buckets(s, stages, buckets, seed)):
            index.setdefault((t, b), []).append(i)
    res = []
    for q in query_sigs:
        cand = set()
        for t, b in enumerate(lsh_buckets(q, stages, buckets, seed)):
            cand.update(index.get((t, b), []))
        scored = []
        for c in sorted(cand):
            d, _ = sketch_distance(np.asarray(q, np.int32), np.asarray(subject_sigs[c], np.int32), width)
            if d <= max_dist:
                scored.append((d, c))
        scored.sort()
        res.append([(c, d) for d, c in scored[:n]])
    return res
