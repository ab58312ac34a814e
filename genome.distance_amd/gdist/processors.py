"""Host-side mirrors of the hot-path processors, driving libgdist.so.

Each function keeps the reference processor's options, defaults, validation
errors and output format, and replaces its per-pair Java loop with whole
row-block / row-query calls on the device:

  fasta_distance   FastaDistanceProcessor  (fastaDist)  FastaDistanceProcessor.java:84-194
  genome_distance  GenomeProcessor         (genomes)    GenomeProcessor.java:74-150
  fasta_reps       FastaDistanceRepsProcessor (fastaReps) FastaDistanceRepsProcessor.java:58-149
  distance_reps    DistanceRepsProcessor   (distReps)   DistanceRepsProcessor.java:140-275
  width_processor  WidthProcessor          (width)      WidthProcessor.java:88-208

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
from .javafmt import java_double, java_format_f
from .kmers import Context, KmerSets, KmerType


class ParseFailureException(ValueError):
    """org.theseed.basic.ParseFailureException (bad command parameters)."""


@dataclasses.dataclass
class Genome:
    """The part of org.theseed.genome.Genome the distance path reads: contig
    DNA (GenomeKmers), protein sequences (ProteinKmers, the `prot` method)
    and the taxonomic lineage rank -> taxon (TaxonDistanceMethod)."""
    id: str
    name: str
    contigs: list[str]
    proteins: list[str] = dataclasses.field(default_factory=list)
    lineage: dict = dataclasses.field(default_factory=dict)

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
    k = kmer_size or kmer_type.getKmerSize()                       # FastaDistanceProcessor.java:95-96
    if k < 2:
        raise ParseFailureException("Kmer size must be at least 2.")   # FastaDistanceProcessor.java:98-99
    if batch < 1:
        raise ParseFailureException("Batch size must be at least 1.")  # FastaDistanceProcessor.java:101-102
    out.write("seq1\tname1\tseq2\tname2\tdistance\n")                 # FastaDistanceProcessor.java:139
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
        raise ParseFailureException("Kmer size cannot be less than 4.")          # GenomeProcessor.java:84-85
    if max_dist <= 0.0 or max_dist > 1.0:
        raise ParseFailureException("Maximum distance must be > 0 and <= 1.")    # GenomeProcessor.java:89-90
    out.write("genome1\tgenome2\tdistance\n")                                    # GenomeProcessor.java:121
    comps = [g for src in others for g in src]
    if not base or not comps:
        return 0
    allg = list(base) + comps
    sets = KmerSets.from_sequences([g.kmer_text() for g in allg], kmer_size, KmerType.DNA, flags, ctx)
    nb = len(base)
    # one rectangle: rows = comparison genomes, cols = base genomes (GenomeProcessor.java:140)
    _, D = sets.matrix((nb, len(allg)), (0, nb), method=method, want_I=False)
    n = 0
    for a, g in enumerate(comps):
        for i, bg in enumerate(base):                                             # GenomeProcessor.java:143-144
            out.write(f"{g.id}\t{bg.id}\t{java_double(D[a, i])}\n")
            n += 1
    return n


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode (UTF-16 code units, int32 wrap-around)."""
    b = s.encode("utf-16-be")
    h = 0
    for i in range(0, len(b), 2):
        h = (31 * h + ((b[i] << 8) | b[i + 1])) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


def java_table_size_for(initial_capacity: int) -> int:
    """java.util.HashMap.tableSizeFor: the power of two >= initial_capacity."""
    cap = 1
    while cap < initial_capacity:
        cap *= 2
    return max(cap, 1)


def java_hashmap_order(keys: Sequence[str], initial_capacity: int = 16) -> list[int]:
    """Iteration order of a java.util.HashMap<String, V> created with
    `new HashMap<>(initial_capacity)` into which `keys` (distinct) were put in
    order: bucket (h ^ h >>> 16) & (cap - 1), cap = tableSizeFor(initial
    capacity), doubled whenever a put takes the size past 0.75 · cap;
    insertion order within a bucket (resizes split bins keeping it). The reps
    processors iterate repMap.values() in this order: distReps creates it with
    capacity 500 (DistanceRepsProcessor.java:175, iterated at :190,238),
    fastaReps with 100 (FastaDistanceRepsProcessor.java:90, iterated at :124).
    Tree bins (>= 8 keys in one bucket of a table >= 64) are not modelled."""
    n = len(keys)
    cap = java_table_size_for(initial_capacity)
    while n > cap * 3 // 4:
        cap *= 2
    def bucket(s):
        h = java_string_hash(s) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)
    return sorted(range(n), key=lambda i: (bucket(keys[i]), i))


#: new HashMap<String, GenomeKmers>(500), DistanceRepsProcessor.java:175
DISTREPS_REPMAP_CAPACITY = 500


def _greedy_host(sets: KmerSets, keys: Sequence[str], max_dist: float) -> list[int]:
    """Pass 1 with the reference's repMap semantics, one row query per set:
    a new representative whose key is already in repMap replaces the old one
    (HashMap.put), keeping that key's slot. Returns the representatives in
    insertion-key order (index of the set each key now maps to)."""
    rep_of_key: dict[str, int] = {}
    for i, key in enumerate(keys):
        reps = list(rep_of_key.values())
        if reps and sets.row_query(i, reps, L.QUERY_ANY_LE, max_dist):
            continue
        rep_of_key[key] = i
    return list(rep_of_key.values())


def _greedy(sets: KmerSets, keys: Sequence[str], max_dist: float) -> list[int]:
    """Pass 1: on the device when keys are unique (gdist_greedy_reps),
    otherwise the host loop with HashMap.put replacement."""
    if len(set(keys)) == len(keys):
        is_rep = sets.greedy_reps(max_dist)
        return [int(i) for i in np.flatnonzero(is_rep)]
    return _greedy_host(sets, keys, max_dist)


def fasta_reps(records: Sequence[FastaRecord], out: TextIO, kmer_size: int = 0, max_dist: float = 0.97,
               kmer_type: KmerType = KmerType.DNA, flags: int = 0, ctx: Context | None = None) -> list[int]:
    """fastaReps (FastaDistanceRepsProcessor.java:111-149): greedy
    representatives in input order; one output line per new representative
    (a repeated label re-enters repMap under its key and is printed again)."""
    k = kmer_size or kmer_type.getKmerSize()
    if k < 2:
        raise ParseFailureException("Kmer size must be at least 2.")           # FastaDistanceRepsProcessor.java:84-85
    out.write("seq\tname\n")                                                  # FastaDistanceRepsProcessor.java:115
    if not records:
        return []
    sets = KmerSets.from_sequences([r.sequence for r in records], k, kmer_type, flags, ctx)
    labels = [r.label for r in records]
    if len(set(labels)) == len(labels):
        reps = _greedy(sets, labels, max_dist)
        printed = reps
    else:
        # replayed on the host to print every put, including replacements
        printed, rep_of_key = [], {}
        for i, key in enumerate(labels):
            cur = list(rep_of_key.values())
            if cur and sets.row_query(i, cur, L.QUERY_ANY_LE, max_dist):
                continue
            rep_of_key[key] = i
            printed.append(i)
        reps = list(rep_of_key.values())
    for i in printed:
        out.write(f"{records[i].label}\t{records[i].comment}\n")            # FastaDistanceRepsProcessor.java:141-144
    return reps


def distance_reps(genomes: Sequence[Genome], kmer_size: int = 9, max_dist: float = 0.97, flags: int = 0,
                  ctx: Context | None = None) -> tuple[str, str, str]:
    """distReps (DistanceRepsProcessor.java:140-275): returns (file name
    prefix, list.tbl text, stats.tbl text). Pass 1 picks representatives in
    input order; pass 2 assigns every genome its closest representative,
    ties to the earlier one in repMap's HashMap iteration order."""
    if kmer_size < 4:
        raise ParseFailureException("Kmer size must be at least 4.")           # DistanceRepsProcessor.java:156-157
    if max_dist <= 0.0 or max_dist >= 1.0:
        raise ParseFailureException("Distance must be strictly between 0 and 1.")  # DistanceRepsProcessor.java:160-161
    prefix = "rep%.4f_K%d" % (max_dist, kmer_size)                              # DistanceRepsProcessor.java:212
    sets = KmerSets.from_sequences([g.kmer_text() for g in genomes], kmer_size, KmerType.DNA, flags, ctx)
    ids = [g.id for g in genomes]
    reps = _greedy(sets, ids, max_dist)                                         # pass 1 (DistanceRepsProcessor.java:185-200)
    rep_set = set(reps)
    # repMap iteration order (keys = genome ids, put in pass-1 order)
    order = java_hashmap_order([ids[r] for r in reps], DISTREPS_REPMAP_CAPACITY)
    ordered_reps = [reps[o] for o in order]
    lines = ["genome_id\tgenome_name\trep_id\trep_name\tdistance"]
    counts: dict[int, int] = {}
    unique = len(set(ids)) == len(ids)
    if unique and reps:
        rank = np.full(len(genomes), len(genomes), dtype=np.int64)
        for pos, r in enumerate(ordered_reps):
            rank[r] = pos
        _, rep_of, rep_d = sets.greedy_reps(max_dist, assign=True, tie_rank=rank)
    for i, g in enumerate(genomes):                                             # pass 2 (DistanceRepsProcessor.java:220-262)
        if i in rep_set:
            r, d = i, 0.0
        elif unique:
            r, d = int(rep_of[i]), float(rep_d[i])
        else:
            pos, d = sets.row_query(i, ordered_reps, L.QUERY_ARGMIN)
            r = ordered_reps[pos]
        rg = genomes[r]
        lines.append(f"{g.id}\t{g.name}\t{rg.id}\t{rg.name}\t{java_double(d)}")
        counts[r] = counts.get(r, 0) + 1
    stats = ["rep_id\trep_name\tsize"]
    for r, c in sorted(counts.items(), key=lambda kv: (-kv[1], genomes[kv[0]].id)):   # sortedCounts (DistanceRepsProcessor.java:268)
        stats.append(f"{genomes[r].id}\t{genomes[r].name}\t{c}")
    return prefix, "\n".join(lines) + "\n", "\n".join(stats) + "\n"


# ----------------------------------------------------------------- width
INVALID_TARGET_SIZE = 2**31 - 1          # Integer.MAX_VALUE, WidthProcessor.java:53


def sketch_sizes(min_size: int, max_size: int, step: int) -> list[int]:
    """SizeList.getSizes(min, max, step) (WidthProcessor.java:104; the class is
    in the absent org.theseed jar): min, min+step, ... up to max (inferred)."""
    return list(range(min_size, max_size + 1, step))


def width_process_group(group_id: str, sets: KmerSets, sizes: Sequence[int], out: TextIO,
                        target_error: float = 0.001) -> int | None:
    """WidthProcessor.ProcessGroup (WidthProcessor.java:153-208): exact
    all-pairs on the device, then per sketch size the sketch all-pairs and the
    relative error |r - s| * 2 / (r + s) over every pair i < j whose distances
    differ, summed in the reference's i-major order; one output line per size.
    Returns the smallest size whose mean error meets the target
    (INVALID_TARGET_SIZE if none), or None for a group with no pair < 1.0."""
    n = len(sets)
    _, D = sets.matrix(upper=True)
    iu = np.triu_indices(n, 1)                      # (i, j) in i-major order
    real = D[iu]
    pairs = int(np.count_nonzero(real < 1.0))
    if pairs == 0:
        return None
    min_good = INVALID_TARGET_SIZE
    for size in sizes:
        sk = sets.sketches(size)
        soff, _ = sk.download()
        dwarves = int(np.count_nonzero(np.diff(soff) < size))
        _, SD = sk.matrix(upper=True)
        s = SD[iu]
        diff = real != s
        err = np.abs(real[diff] - s[diff]) * 2.0 / (real[diff] + s[diff])
        total = float(np.cumsum(err)[-1]) if err.size else 0.0     # sequential, as `total += error`
        max_err = 0.0
        if err.size:
            m = float(np.max(err))
            max_err = m if m > 0.0 else 0.0
        mean = total / pairs
        out.write(f"{group_id}\t{size:8d}\t{pairs:8d}\t{dwarves:8d}\t{java_format_f(mean, 8, 4)}\t"
                  f"{java_format_f(max_err, 8, 4)}\n")
        if size < min_good and mean <= target_error:
            min_good = size
    return min_good


def width_processor(rows: Iterable[tuple[str, str]], min_size: int, max_size: int, out: TextIO,
                    step: int = 10, max_group: int = 1000, target_error: float = 0.001, kmer_size: int = 8,
                    ctx: Context | None = None) -> int:
    """WidthProcessor (width): `rows` are (group id, protein sequence) in input
    order; consecutive rows of one group form a group, split at max_group
    (WidthProcessor.java:117-131). Validation as validateParms
    (WidthProcessor.java:88-106). Returns the target sketch size (the largest
    per-group minimum, INVALID_TARGET_SIZE when some group had none)."""
    if min_size > max_size:
        raise ParseFailureException("Minimum sketch size cannot be larger than maximum.")
    if step <= 0:
        raise ParseFailureException("Step size must be greater than 0.")
    if max_group < 10:
        raise ParseFailureException("Maximum group size must be 10 or greater.")
    if target_error > 0.1 or target_error <= 0.0:
        raise ParseFailureException("Target error must be > 0 and < 0.1.")
    sizes = sketch_sizes(min_size, max_size, step)
    target = min_size
    out.write("Group\tSize\tPairs\tDwarves\tMean E\tMax E\n")

    def flush(gid, prots):
        nonlocal target
        sets = KmerSets.from_sequences(prots, kmer_size, KmerType.PROT, 0, ctx)
        good = width_process_group(gid, sets, sizes, out, target_error)
        if good is not None and good > target:
            target = good

    group_id, prots = "", []
    for gid, seq in rows:
        if gid != group_id or len(prots) >= max_group:
            if prots:
                flush(group_id, prots)
            group_id, prots = gid, []
        prots.append(seq)
    if prots:
        flush(group_id, prots)
    return target
