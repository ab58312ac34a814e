"""CPU: every `Name.java:N[-M]` citation in the product, oracle and host code
resolves against the reference sources (the file exists, every cited line is
inside it), and where a cited line carries a message or output literal, the
literal is on the cited lines. Skips when /root/reference is absent (the GPU
box never has it)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src/main/java"
SCANNED = ["include", "oracle", "genome.distance_amd/gdist", "genome.distance_amd/csrc", "tests",
           "INTEGRATION.md", "DESIGN.md", "bench.py", "__graft_entry__.py"]
CITE = re.compile(r"([A-Za-z]+\.java):(\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")
LITERAL = re.compile(r'"((?:[^"\\]|\\.){12,})"')


def _ref_files():
    out = {}
    for p in glob.glob(os.path.join(REF, "**", "*.java"), recursive=True):
        with open(p, errors="replace") as f:
            out[os.path.basename(p)] = f.read().split("\n")
    return out


def _sources():
    for entry in SCANNED:
        p = os.path.join(ROOT, entry)
        if os.path.isfile(p):
            yield p
            continue
        for dirpath, _, files in os.walk(p):
            for fn in files:
                if fn.endswith((".py", ".h", ".hip", ".hpp", ".c", ".md")):
                    yield os.path.join(dirpath, fn)


def _ranges(spec):
    for part in spec.split(","):
        a, _, b = part.strip().partition("-")
        yield int(a), int(b or a)


def _citations():
    for path in _sources():
        with open(path, errors="replace") as f:
            for ln, line in enumerate(f, 1):
                for m in CITE.finditer(line):
                    yield path, ln, line, m.group(1), list(_ranges(m.group(2)))


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent")
def test_citations_resolve():
    ref = _ref_files()
    bad, n = [], 0
    for path, ln, _, name, ranges in _citations():
        n += 1
        rel = os.path.relpath(path, ROOT)
        if name not in ref:
            bad.append(f"{rel}:{ln}: {name} is not a reference file")
            continue
        nlines = len(ref[name])
        for a, b in ranges:
            if not (1 <= a <= b <= nlines):
                bad.append(f"{rel}:{ln}: {name}:{a}-{b} outside its {nlines} lines")
    assert n > 50, "citation scan found too few citations"
    assert not bad, "\n".join(bad)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent")
def test_cited_literals_are_on_the_cited_lines():
    """A host-code line that raises a reference message or writes a reference
    header, and cites the reference line it follows, must cite the line that
    holds that text (catches citations shifted to a wrong but existing line)."""
    ref = _ref_files()
    bad, checked = [], 0
    for path, ln, line, name, ranges in _citations():
        if not path.endswith(".py") or name not in ref or not ("raise " in line or ".write(" in line):
            continue
        lits = [x for x in LITERAL.findall(line) if not x.startswith(("{", "%"))]
        if not lits:
            continue
        text = "\n".join("\n".join(ref[name][a - 1:b]) for a, b in ranges)
        for lit in lits:
            probe = lit.split("{")[0].replace("\\n", "")[:40]
            if len(probe) < 8:
                continue
            checked += 1
            if probe not in text:
                bad.append(f"{os.path.relpath(path, ROOT)}:{ln}: {lit!r} not on {name}:{ranges}")
    assert checked >= 8, f"only {checked} cited literals found"
    assert not bad, "\n".join(bad)
