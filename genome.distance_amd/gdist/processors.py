"""Host-side mirrors of the hot-path processors, driving libgdist.so.

Each function keeps the reference processor's options, defaults, validation
errors and output format, and replaces its per-pair Java loop with whole
row-block / row-query calls on the device:

  fasta_distance   FastaDistanceProcessor  (fastaDist)  FastaDistanceProcessor.java:84-194
  genome_distance  GenomeProcessor         (genomes)    GenomeProcessor.java:270-346
  fasta_reps       FastaDistanceRepsProcessor (fastaReps) FastaDistanceRepsProcessor.java:58-149
  distance_reps    DistanceRepsProcessor   (distReps)   DistanceRepsProcessor.java:350-485

Output rows are emitted in (row, column) order; the reference's fastaDist
order is nondeterministic (rows run in parallel, FastaDistanceProcessor.java:157,188),
so consumers compare those outputs as sets of lines.
"""
from __future__ import annotations

import dataclasses
from typing import Iterable, Iterator, Sequence, TextIO

import numpy as np

from . import _lib as L
from .fasta import Sequence as FastaRecord
from .javafmt import java_double
from .kmers import Context, KmerSets, KmerType


class ParseFailureException(ValueError):
    """org.theseed.basic.ParseFailureException (bad command parameters)."""


@dataclasses.dataclass
class Genome:
    """The part of org.theseed.genome.Genome the distance path reads."""
    id: str
    name: str
    contigs: list[str]

    def kmer_text(self) -> bytes:
        # contigs joined by the 0x00 separator: one set, no kmer spans contigs
        return b"\0".join(c.encode("latin-1") for c in self.contigs)


def _row_blocks(n: int, block: int) -> Iterator[tuple[int, int]]:
    for r0 in range(0, n, block):
        yield r0, min(n, r0 + block)


def fasta_distance(records: Sequence[FastaRecord], out: TextIO, kmer_size: int = 0, batch: int = 20,
                   kmer_type: KmerType = KmerType.DNA, flags: int = 0, method: int = L.METHOD_AUTO,
                   ctx: Context | None = None, row_block: int = 1024) -> int:
    """fastaDist: N×N upper triangle of kmer distances over FASTA records."""
    k = kmer_size or kmer_type.getKmerSize()                       # :95-96
    if k < 2:
        raise ParseFailureException("Kmer size must be at least 2.")   # :98-99
    if batch < 1:
        raise ParseFailureException("Batch size must be at least 1.")  # :101-102
    out.write("seq1\tname1\tseq2\tname2\tdistance\n")                 # :139
    n = len(records)
    if n < 2:
        return 0
    sets = KmerSets.from_sequences([r.sequence for r in records], k, kmer_type, flags, ctx)
    if method == L.METHOD_BITSET:
        sets.build_bitsets()
    pairs = 0
    for r0, r1 in _row_blocks(n, row_block):
        _, D = sets.matrix((r0, r1), (0, n), upper=True, method=method, want_I=False)
        for a in range(r0, r1):
            ra = records[a]
            row = D[a - r0]
            for j in range(a + 1, n):
                rb = records[j]
                out.write(f"{ra.label}\t{ra.comment}\t{rb.label}\t{rb.comment}\t{java_double(row[j])}\n")
                pairs += 1
    return pairs


def genome_distance(base: Sequence[Genome], others: Sequence[Sequence[Genome]], out: TextIO,
                    kmer_size: int = 21, max_dist: float = 0.9, flags: int = 0,
                    method: int = L.METHOD_AUTO, ctx: Context | None = None) -> int:
    """genomes: every comparison genome against every base genome."""
    if kmer_size < 4:
        raise ParseFailureException("Kmer size cannot be less than 4.")          # GenomeProcessor.java:280-281
    if max_dist <= 0.0 or max_dist > 1.0:
        raise ParseFailureException("Maximum distance must be > 0 and <= 1.")    # :285-286
    out.write("genome1\tgenome2\tdistance\n")                                    # :317
    comps = [g for src in others for g in src]
    if not base or not comps:
        return 0
    allg = list(base) + comps
    sets = KmerSets.from_sequences([g.kmer_text() for g in allg], kmer_size, KmerType.DNA, flags, ctx)
    nb = len(base)
    # one rectangle: rows = comparison genomes, cols = base genomes (:336)
    _, D = sets.matrix((nb, len(allg)), (0, nb), method=method, want_I=False)
    n = 0
    for a, g in enumerate(comps):
        for i, bg in enumerate(base):                                             # :339-341
            out.write(f"{g.id}\t{bg.id}\t{java_double(D[a, i])}\n")
            n += 1
    return n


def fasta_reps(records: Sequence[FastaRecord], out: TextIO, kmer_size: int = 0, max_dist: float = 0.97,
               kmer_type: KmerType = KmerType.DNA, flags: int = 0, ctx: Context | None = None) -> list[int]:
    """fastaReps: greedy representatives in input order (sequential early exit)."""
    k = kmer_size or kmer_type.getKmerSize()
    if k < 2:
        raise ParseFailureException("Kmer size must be at least 2.")           # :96-97
    out.write("seq\tname\n")                                                    # :121
    if not records:
        return []
    sets = KmerSets.from_sequences([r.sequence for r in records], k, kmer_type, flags, ctx)
    reps: list[int] = []
    for i, r in enumerate(records):
        # any(rep distance <= maxDist) — order-independent boolean (:124-133)
        if reps and sets.row_query(i, reps, L.QUERY_ANY_LE, max_dist):
            continue
        reps.append(i)
        out.write(f"{r.label}\t{r.comment}\n")                                  # :139-141
    return reps


def distance_reps(genomes: Sequence[Genome], kmer_size: int = 9, max_dist: float = 0.97, flags: int = 0,
                  ctx: Context | None = None) -> tuple[str, str, str]:
    """distReps: returns (file name prefix, list.tbl text, stats.tbl text)."""
    if kmer_size < 4:
        raise ParseFailureException("Kmer size must be at least 4.")           # :366-367
    if max_dist <= 0.0 or max_dist >= 1.0:
        raise ParseFailureException("Distance must be strictly between 0 and 1.")  # :370-371
    prefix = "rep%.4f_K%d" % (max_dist, kmer_size)                              # :422
    sets = KmerSets.from_sequences([g.kmer_text() for g in genomes], kmer_size, KmerType.DNA, flags, ctx)
    reps: list[int] = []
    for i in range(len(genomes)):                                               # pass 1 (:395-411)
        if reps and sets.row_query(i, reps, L.QUERY_ANY_LE, max_dist):
            continue
        reps.append(i)
    rep_set = set(reps)
    lines = ["genome_id\tgenome_name\trep_id\trep_name\tdistance"]
    counts: dict[int, int] = {}
    for i, g in enumerate(genomes):                                             # pass 2 (:430-470)
        if i in rep_set:
            r, d = i, 0.0
        else:
            pos, d = sets.row_query(i, reps, L.QUERY_ARGMIN)
            r = reps[pos]
        rg = genomes[r]
        lines.append(f"{g.id}\t{g.name}\t{rg.id}\t{rg.name}\t{java_double(d)}")
        counts[r] = counts.get(r, 0) + 1
    stats = ["rep_id\trep_name\tsize"]
    for r, c in sorted(counts.items(), key=lambda kv: (-kv[1], genomes[kv[0]].id)):   # sortedCounts (:478)
        stats.append(f"{genomes[r].id}\t{genomes[r].name}\t{c}")
    return prefix, "\n".join(lines) + "\n", "\n".join(stats) + "\n"
