"""Pure-Python string-set restatement of the reference kmer-distance path.

TEST INFRASTRUCTURE ONLY (fixture generator / cross-check for the C oracle).
PARITY UNPINNED: the reference's kmer classes live in the un-vendored
org.theseed:sequence:1.0.0 module (pom.xml:46-49) and no JVM exists here, so
this restatement follows the in-repo call sites and the packing spec in
include/gdist.h. It deliberately works on Python `str` kmers in `set`s — the
shape of the Java HashSet<String> — and never on packed codes, so it is an
independent check of oracle/gdist_oracle.c's code packing and merge logic.
"""
from __future__ import annotations

import math
import struct

DNA, PROT = 0, 1
STRAND_BOTH, STRAND_FWD, STRAND_CANON = 0x0, 0x1, 0x2
AMBIG_DEFAULT, AMBIG_SKIP, AMBIG_KEEP = 0x0, 0x4, 0x8
NO_CASE_FOLD = 0x10
EMPTY_NAN = 0x400
SKETCH_JACCARD = 0x800

_STANDARD_AA = set("ACDEFGHIKLMNPQRSTVWY")
_COMP = {"A": "T", "T": "A", "C": "G", "G": "C", "N": "N", "R": "Y", "Y": "R"}


def _ambig_skip(kind: int, flags: int) -> bool:
    m = flags & 0xC
    if m == AMBIG_SKIP:
        return True
    if m == AMBIG_KEEP:
        return False
    return kind == DNA


def _fold(s: str) -> str:
    return "".join(chr(ord(c) - 32) if "a" <= c <= "z" else c for c in s)


def kmer_set(seq: str, k: int, kind: int = DNA, flags: int = 0) -> set[str]:
    """KmerType.createKmers(seq, k) — FastaDistanceProcessor.java:153,184.

    "\0" separates pieces (contigs of one genome): no kmer spans it."""
    if "\0" in seq:
        _check_encodable(seq.replace("\0", ""), k, kind, flags)
        out: set[str] = set()
        for piece in seq.split("\0"):
            out |= kmer_set(piece, k, kind, flags)
        return out
    if kind == DNA or not (flags & NO_CASE_FOLD):
        seq = _fold(seq)
    skip = _ambig_skip(kind, flags)
    strand = flags & 0x3
    _check_encodable(seq, k, kind, flags)
    out: set[str] = set()
    for i in range(len(seq) - k + 1):
        w = seq[i:i + k]
        if skip:
            ok = all(c in "ACGT" for c in w) if kind == DNA else all(c in _STANDARD_AA for c in w)
            if not ok:
                continue
        if kind == DNA and strand != STRAND_FWD:
            rc = "".join(_COMP.get(c, c) for c in reversed(w))
            if strand == STRAND_CANON:
                out.add(min(w, rc))
            else:
                out.add(w)
                out.add(rc)
        else:
            out.add(w)
    return out


def _check_encodable(seq: str, k: int, kind: int, flags: int) -> None:
    """Packing spec: a sequence holding a char the code cannot represent is
    rejected as a whole (gdist.h: EINVAL), whatever k is."""
    if kind == DNA or not (flags & NO_CASE_FOLD):
        seq = _fold(seq)
    skip = _ambig_skip(kind, flags)
    if kind == DNA and not skip and any(c not in "ACGNRTY" for c in seq):
        raise ValueError("unencodable DNA char in keep mode")
    if kind == PROT and k > 8 and any(
            not (c == "*" or "A" <= c <= "Z") for c in seq if not (skip and c not in _STANDARD_AA)):
        raise ValueError("unencodable protein char for k > 8")


def encode(kmer: str, kind: int = DNA, flags: int = 0) -> int:
    """Packing spec of include/gdist.h (order-preserving, injective)."""
    k = len(kmer)
    if kind == DNA:
        alpha = "ACGT" if _ambig_skip(kind, flags) else "ACGNRTY"
        bits = 2 if len(alpha) == 4 else 3
        syms = [alpha.index(c) for c in kmer]
    else:
        if k <= 8:
            bits, syms = 8, [ord(c) for c in kmer]
        else:
            bits = 5
            if any(not (c == "*" or "A" <= c <= "Z") for c in kmer):
                raise ValueError("unencodable protein char for k > 8")
            syms = [0 if c == "*" else 1 + ord(c) - ord("A") for c in kmer]
    code = 0
    for s in syms:
        code = (code << bits) | s
    return code


def distance(inter: int, na: int, nb: int, flags: int = 0) -> float:
    """SequenceKmers.distance (inferred Java expression)."""
    if inter > 0:
        return 1.0 - inter / float(na + nb - inter)
    if na + nb == 0 and flags & EMPTY_NAN:
        return float("nan")
    return 1.0


def set_distance(a: set[str], b: set[str], flags: int = 0) -> float:
    return distance(len(a & b), len(a), len(b), flags)


def java_double_str(d: float) -> str:
    """Java Double.toString (JDK 19+ algorithm, JDK 21 per pom.xml:17)."""
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    digits, e = _digits_exp(repr(d))   # shortest round-trip digits
    if len(digits) == 1:
        digits, e = _digits_exp("%.1e" % d)
    digits = digits.rstrip("0") or "0"
    neg = d < 0
    a = abs(d)
    if 1e-3 <= a < 1e7:
        if e >= 0:
            ip = "".join(digits[i] if i < len(digits) else "0" for i in range(e + 1))
            fp = digits[e + 1:] or "0"
            s = ip + "." + fp
        else:
            s = "0." + "0" * (-e - 1) + digits
    else:
        s = digits[0] + "." + (digits[1:] or "0") + "E" + str(e)
    return ("-" if neg else "") + s


def _digits_exp(s: str) -> tuple[str, int]:
    s = s.lstrip("-")
    if "e" in s or "E" in s:
        m, _, x = s.lower().partition("e")
        e = int(x)
    else:
        m, e = s, 0
    if "." in m:
        ip, fp = m.split(".")
    else:
        ip, fp = m, ""
    # normalise to d.ddd x 10^e
    allds = ip + fp
    e += len(ip) - 1
    stripped = allds.lstrip("0")
    e -= len(allds) - len(stripped)
    return stripped or "0", e


def murmur3_32(data: bytes, seed: int = 0) -> int:
    """MurmurHash3_x86_32, returned as a Java signed int."""
    c1, c2 = 0xCC9E2D51, 0x1B873593
    h = seed & 0xFFFFFFFF
    n = len(data) // 4
    for i in range(n):
        k = struct.unpack_from("<I", data, 4 * i)[0]
        k = (k * c1) & 0xFFFFFFFF
        k = ((k << 15) | (k >> 17)) & 0xFFFFFFFF
        k = (k * c2) & 0xFFFFFFFF
        h ^= k
        h = ((h << 13) | (h >> 19)) & 0xFFFFFFFF
        h = (h * 5 + 0xE6546B64) & 0xFFFFFFFF
    tail = data[4 * n:]
    k1 = 0
    if len(tail) >= 3:
        k1 ^= tail[2] << 16
    if len(tail) >= 2:
        k1 ^= tail[1] << 8
    if len(tail) >= 1:
        k1 ^= tail[0]
        k1 = (k1 * c1) & 0xFFFFFFFF
        k1 = ((k1 << 15) | (k1 >> 17)) & 0xFFFFFFFF
        k1 = (k1 * c2) & 0xFFFFFFFF
        h ^= k1
    h ^= len(data)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h - (1 << 32) if h & 0x80000000 else h


def sketch(kmers: set[str], width: int) -> list[int]:
    """SequenceKmers.hashSet(width) restatement (SketchProcessor.java:88)."""
    hs = sorted({murmur3_32(x.encode("latin-1")) for x in kmers})
    return hs[:width]


def sketch_distance(a: list[int], b: list[int], width: int, flags: int = 0) -> tuple[float, int]:
    """Sketch.distance restatement (WidthProcessor.java:185); returns (d, common)."""
    if flags & SKETCH_JACCARD:
        common = len(set(a) & set(b))
        return distance(common, len(a), len(b), flags), common
    union = sorted(set(a) | set(b))[:width]
    sa, sb = set(a), set(b)
    common = sum(1 for x in union if x in sa and x in sb)
    taken = len(union)
    if common > 0:
        return 1.0 - common / float(taken), common
    if taken == 0 and flags & EMPTY_NAN:
        return float("nan"), 0
    return 1.0, 0
