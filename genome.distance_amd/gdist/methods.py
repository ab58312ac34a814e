"""DistanceMethod / Measurer plugin mirror and the `methods` command driver.

Reference: MethodTableProcessor.java (the `methods` subcommand) drives the
plugin API of the un-vendored org.theseed:distance module:
  DistanceMethod.loadRoles(roleFile)                   MethodTableProcessor.java:168
  DistanceMethod.create(type), parseParmString(parms)  MethodTableProcessor.java:175-182
  toString() as the output column header               MethodTableProcessor.java:243
  getMeasurer(genome1), once per first genome          MethodTableProcessor.java:261-265,397-407
  getDistance(measurer, genome2) from ForkJoin threads MethodTableProcessor.java:275
  close()                                              MethodTableProcessor.java:304-306
`method_table` restates runPipeline (MethodTableProcessor.java:234-308) with
its previous-results reuse (:186-221, :270-272, :319-332), header, Java
`Double.toString` rows (:283-289) and correlation statistics (:339-378).

GPU form: a Measurer keeps its genome's kmer text. The pair list is grouped
by id1 (GenomePairList.prepare, :240), so the driver asks each method for the
whole group at once (`prefetch`: ONE pack of the first genome with the
group's second genomes and one device row query per method) and the per-pair
`getDistance` calls — issued concurrently, one thread per method, as :275
does — are answered from that row without a lock on the method. A
`getDistance` on a genome outside a prefetched group is one device call of
its own (pack of the two genomes + a one-column row query).

What the un-vendored module decides and this restatement infers (parity
unpinned): the kmer methods' type names and parameter syntax
("K=8"), their toString ("PROT_K8"), GenomePairList's grouping order (first
appearance of id1, pairs of a group in input order), TaxonDistanceMethod's
grouping level (deepest shared lineage rank) and CorrelationVariance's
variation / IQR (mean |d1 - d2| and the interquartile range of d1 - d2).
"""
from __future__ import annotations

import concurrent.futures as cf
import math
import threading
from typing import Iterable, Mapping, Sequence, TextIO

import numpy as np

from . import _lib as L
from .javafmt import java_double, java_format_f
from .kmers import Context, KmerSets, KmerType
from .processors import Genome, ParseFailureException


class Measurer:
    """A genome prepared for repeated distance measurements: its kmer text,
    built once (getMeasurer, MethodTableProcessor.java:397-407), and the row
    of distances of its id1 group once prefetched."""

    def __init__(self, method: "DistanceMethod", genome: Genome):
        self.method = method
        self.genome = genome
        self.text = method.kmer_text(genome)
        self._row: dict[str, float] = {}      # prefetched distances by second genome id
        self._lock = threading.Lock()         # guards _row only, never a device call


class DistanceMethod:
    """Base of the plugin; subclasses register a type name."""
    _registry: dict[str, type] = {}
    type_name = "?"
    _roles: set[str] | None = None

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        DistanceMethod._registry[cls.type_name.lower()] = cls

    @staticmethod
    def create(type_name: str, ctx: Context | None = None) -> "DistanceMethod":
        cls = DistanceMethod._registry.get(type_name.lower())
        if cls is None:
            raise ParseFailureException(f"Invalid distance method type \"{type_name}\".")
        return cls(ctx)

    @staticmethod
    def loadRoles(path) -> None:
        """Role definitions (roles.in.subsystems); kmer methods do not use them."""
        roles = set()
        with open(path) as f:
            for line in f:
                bits = line.rstrip("\n").split("\t")
                if bits and bits[0]:
                    roles.add(bits[0])
        DistanceMethod._roles = roles

    def __init__(self, ctx: Context | None = None):
        self.ctx = ctx or Context.default()

    def parseParmString(self, parms: str) -> None:
        raise NotImplementedError

    def getMeasurer(self, genome: Genome) -> Measurer:
        return Measurer(self, genome)

    def getDistance(self, measurer: Measurer, genome: Genome) -> float:
        """Thread-safe (the reference calls it from ForkJoin threads, :275):
        a prefetched group's distance is a dictionary read; any other pair is
        one device call of its own (no lock held across it: the library's
        context serialises only its own device work)."""
        with measurer._lock:
            d = measurer._row.get(genome.id)
        if d is not None:
            return d
        return self.getDistances(measurer, [genome])[0]

    def getDistances(self, measurer: Measurer, genomes: Sequence[Genome]) -> list[float]:
        """Batched getDistance: the measurer's genome and `genomes` packed in
        ONE call (set 0 = the measurer's) and one device row query of set 0
        against the rest: no copy of the measurer's set, no method-wide lock."""
        if not genomes:
            return []
        sets = KmerSets.from_sequences([measurer.text] + [self.kmer_text(g) for g in genomes], self.k,
                                       self.kmer_type, self.flags, self.ctx)
        try:
            d = sets.row_query(0, range(1, 1 + len(genomes)), L.QUERY_ALL)
        finally:
            sets.free()
        return [float(x) for x in d]

    def prefetch(self, measurer: Measurer, genomes: Sequence[Genome]) -> None:
        """Distances of a whole id1 group in one batched query, kept on the
        measurer for getDistance (GenomePairList.prepare groups pairs by id1,
        MethodTableProcessor.java:240,261-275)."""
        with measurer._lock:
            todo = [g for g in genomes if g.id not in measurer._row]
        uniq = list({g.id: g for g in todo}.values())
        row = dict(zip((g.id for g in uniq), self.getDistances(measurer, uniq)))
        with measurer._lock:
            measurer._row.update(row)

    def close(self) -> None:
        pass


class _KmerMethod(DistanceMethod):
    kmer_type = KmerType.DNA
    default_k = 21

    def __init__(self, ctx=None):
        super().__init__(ctx)
        self.k = self.default_k
        self.flags = 0

    def parseParmString(self, parms: str) -> None:
        for tok in (parms or "").replace(",", " ").split():
            key, _, val = tok.partition("=")
            if key.upper() in ("K", "KMER", "KMERSIZE"):
                try:
                    self.k = int(val)
                except ValueError:
                    raise ParseFailureException(f"Invalid kmer size \"{val}\" for {self.type_name}.") from None
            else:
                raise ParseFailureException(f"Invalid parameter \"{tok}\" for {self.type_name}.")
        if self.k < 2:
            raise ParseFailureException("Kmer size must be at least 2.")

    def __str__(self) -> str:
        return f"{self.type_name.upper()}_K{self.k}"


class DnaKmerMethod(_KmerMethod):
    """Contig DNA kmer distance (GenomeKmers, GenomeProcessor.java:109,140)."""
    type_name = "kmer"

    def kmer_text(self, g: Genome) -> bytes:
        return g.kmer_text()


class ProteinKmerMethod(_KmerMethod):
    """Protein kmer distance over a genome's proteins (ProteinKmers, k=8 default,
    ProteinKmerReader.java:64,92,101); the proteins form one set, no kmer
    spans two proteins."""
    type_name = "prot"
    kmer_type = KmerType.PROT
    default_k = 8

    def kmer_text(self, g: Genome) -> bytes:
        return b"\0".join(p.encode("latin-1") for p in (g.proteins or []))


class TaxonDistanceMethod:
    """TaxonDistanceMethod's grouping level (MethodTableProcessor.java:230,280-281):
    the most specific rank at which the two genomes' lineages agree, "none"
    when they share no ranked taxon (inferred; the class is un-vendored)."""
    RANKS = ("superkingdom", "phylum", "class", "order", "family", "genus", "species")

    class Analysis:
        def __init__(self, genome: Genome):
            self.lineage = dict(getattr(genome, "lineage", None) or {})

    def getGroupingLevel(self, a1: "TaxonDistanceMethod.Analysis", a2: "TaxonDistanceMethod.Analysis") -> str:
        for rank in reversed(self.RANKS):
            t1, t2 = a1.lineage.get(rank), a2.lineage.get(rank)
            if t1 is not None and t1 == t2:
                return rank
        return "none"

    def close(self) -> None:
        pass


# ---------------------------------------------------------------- the driver
def read_method_file(lines: Iterable[str], ctx: Context | None = None) -> list[DistanceMethod]:
    """The method list (MethodTableProcessor.java:172-183): a header line, then
    tab-separated (type, parameter string) per method."""
    it = iter(lines)
    next(it, None)                                     # TabbedLineReader: header
    methods = []
    for line in it:
        line = line.rstrip("\n")
        if not line:
            continue
        cols = line.split("\t")
        m = DistanceMethod.create(cols[0], ctx)
        m.parseParmString(cols[1] if len(cols) > 1 else "")
        methods.append(m)
    return methods


def _find_field(labels: Sequence[str], name: str) -> int:
    """TabbedLineReader.findField: a column name, or a 1-based index."""
    if name in labels:
        return list(labels).index(name)
    if name.isdigit() and 1 <= int(name) <= len(labels):
        return int(name) - 1
    raise IOError(f"Field \"{name}\" not found in input.")


def read_pairs(lines: Iterable[str], col1: str = "1", col2: str = "2") -> list[tuple[str, str]]:
    """validatePipeInput (MethodTableProcessor.java:149-163)."""
    it = iter(lines)
    head = next(it, "").rstrip("\n").split("\t")
    i1, i2 = _find_field(head, col1), _find_field(head, col2)
    out = []
    for line in it:
        line = line.rstrip("\n")
        if line:
            cols = line.split("\t")
            out.append((cols[i1], cols[i2]))
    return out


def load_previous(lines: Iterable[str], methods: Sequence[DistanceMethod]) -> dict[tuple[str, str], list[float]]:
    """Previous results (MethodTableProcessor.java:186-221): the columns after
    tax_group must be exactly the methods' toString() headers."""
    it = iter(lines)
    labels = next(it, "").rstrip("\n").split("\t")
    method0 = _find_field(labels, "tax_group") + 1
    n = len(methods)
    if method0 + n != len(labels):
        raise IOError("Previous-results file has the wrong number of columns for this method configuration.")
    for i, m in enumerate(methods):
        if labels[i + method0] != str(m):
            raise IOError(f"Method {i} does not match previous-results file.")
    id1c, id2c = _find_field(labels, "id1"), _find_field(labels, "id2")
    old = {}
    for line in it:
        line = line.rstrip("\n")
        if not line:
            continue
        cols = line.split("\t")
        old[(cols[id1c], cols[id2c])] = [float(cols[method0 + i]) for i in range(n)]   # Double.parseDouble
    return old


def group_pairs(pairs: Sequence[tuple[str, str]]) -> list[tuple[str, list[str]]]:
    """GenomePairList.prepare (:240): pairs grouped by id1 (first appearance),
    each group's second genomes in input order (inferred)."""
    groups: dict[str, list[str]] = {}
    for a, b in pairs:
        groups.setdefault(a, []).append(b)
    return list(groups.items())


def method_table(pairs: Sequence[tuple[str, str]], methods: Sequence[DistanceMethod], genomes: Mapping[str, Genome],
                 out: TextIO, stats: TextIO | None = None,
                 previous: Mapping[tuple[str, str], Sequence[float]] | None = None,
                 threads: int = 0, batch: bool = True) -> dict:
    """runPipeline (MethodTableProcessor.java:234-308). `genomes` is the
    genome source (id -> Genome); `previous` the map load_previous returns.
    Per pair the methods run concurrently (:275, one thread per method);
    with batch=True each method first prefetches its id1 group in one
    device row query. Returns counters (pairs, computed, reused)."""
    missing = sorted({x for p in pairs for x in p if x not in genomes})
    if missing:                                        # checkGenomes (:426-433)
        raise IOError("The following genomes are missing from the sources: " + ", ".join(missing))
    out.write("id1\tname1\tid2\tname2\ttax_group\t" + "\t".join(str(m) for m in methods) + "\n")   # :242-243
    tax = TaxonDistanceMethod()
    nm = len(methods)
    dist_list: list[list[float]] = []
    counts = {"pairs": 0, "computed": 0, "reused": 0}
    pool = cf.ThreadPoolExecutor(max(1, threads or nm))
    try:
        for id1, ids2 in group_pairs(pairs):
            g1 = genomes[id1]
            measurers = [m.getMeasurer(g1) for m in methods]          # getMeasurers (:397-407)
            a1 = TaxonDistanceMethod.Analysis(g1)
            todo = [genomes[b] for b in ids2 if previous is None or (id1, b) not in previous]
            if batch and todo:
                list(pool.map(lambda i: methods[i].prefetch(measurers[i], todo), range(nm)))
            for id2 in ids2:
                g2 = genomes[id2]
                if previous is not None and (id1, id2) in previous:   # checkPrevious (:319-332)
                    distances = [float(x) for x in previous[(id1, id2)]]
                    counts["reused"] += 1
                else:
                    distances = list(pool.map(lambda i: methods[i].getDistance(measurers[i], g2), range(nm)))
                    counts["computed"] += 1
                dist_list.append(distances)
                group = tax.getGroupingLevel(a1, TaxonDistanceMethod.Analysis(g2))
                line = f"{id1}\t{g1.name}\t{id2}\t{g2.name}\t{group}"           # :283-287
                out.write(line + "".join("\t" + java_double(d) for d in distances) + "\n")
                counts["pairs"] += 1
        if stats is not None and dist_list:
            write_statistics(stats, methods, dist_list)
    finally:
        pool.shutdown()
        for m in methods:                              # :304-306
            m.close()
        tax.close()
    return counts


def _ranks(x: np.ndarray) -> np.ndarray:
    """NaturalRanking with TiesStrategy.AVERAGE (commons-math SpearmansCorrelation)."""
    order = np.argsort(x, kind="mergesort")
    r = np.empty(len(x), np.float64)
    xs = x[order]
    i = 0
    while i < len(x):
        j = i
        while j + 1 < len(x) and xs[j + 1] == xs[i]:
            j += 1
        r[order[i:j + 1]] = (i + j) / 2.0 + 1.0
        i = j + 1
    return r


def _pearson(a: np.ndarray, b: np.ndarray) -> float:
    if len(a) < 2:
        return math.nan
    da, db = a - a.mean(), b - b.mean()
    den = math.sqrt(float((da * da).sum()) * float((db * db).sum()))
    return float((da * db).sum()) / den if den > 0 else math.nan


def _kendall_tau_b(a: np.ndarray, b: np.ndarray) -> float:
    n = len(a)
    conc = disc = ta = tb = 0
    for i in range(n):
        for j in range(i + 1, n):
            x, y = np.sign(a[i] - a[j]), np.sign(b[i] - b[j])
            if x == 0 and y == 0:
                continue
            if x == 0:
                ta += 1
            elif y == 0:
                tb += 1
            elif x == y:
                conc += 1
            else:
                disc += 1
    den = math.sqrt((conc + disc + ta) * (conc + disc + tb))
    return (conc - disc) / den if den > 0 else math.nan


def write_statistics(out: TextIO, methods: Sequence[DistanceMethod], dist_list: Sequence[Sequence[float]]) -> None:
    """writeStatistics (MethodTableProcessor.java:339-378): every method pair in
    both directions, sorted by (method1, method2), "%8.4f" columns."""
    D = np.asarray(dist_list, np.float64)
    out.write("method1\tmethod2\tPearson\tKendall\tSpearman\tvariation\tIQR\n")
    lines = {}
    names = [str(m) for m in methods]
    for i in range(len(methods)):
        for j in range(i + 1, len(methods)):
            a, b = D[:, i], D[:, j]
            p, k = _pearson(a, b), _kendall_tau_b(a, b)
            s = _pearson(_ranks(a), _ranks(b))
            diff = a - b
            tm = float(np.mean(np.abs(diff)))
            iqr = float(np.percentile(diff, 75) - np.percentile(diff, 25))
            vals = "\t".join(java_format_f(v, 8, 4) for v in (p, k, s, tm, iqr))
            lines[(names[i], names[j])] = f"{names[i]}\t{names[j]}\t{vals}"
            lines[(names[j], names[i])] = f"{names[j]}\t{names[i]}\t{vals}"
    for key in sorted(lines):
        out.write(lines[key] + "\n")
