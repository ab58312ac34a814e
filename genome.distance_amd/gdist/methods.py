"""DistanceMethod / Measurer plugin mirror (org.theseed.genome.distance.methods).

The reference's `methods` command (MethodTableProcessor.java:166-308) drives
this API: DistanceMethod.create(type) and parseParmString(parms) per line of
the method file (MethodTableProcessor.java:175-182), toString() as the output
column header (MethodTableProcessor.java:243), getMeasurer(genome1) once per
first genome (MethodTableProcessor.java:261-265,397-407),
getDistance(measurer, genome2) from ForkJoin threads
(MethodTableProcessor.java:275) and close() (MethodTableProcessor.java:304-306). The method classes themselves live in the un-vendored
org.theseed:distance module; the kmer methods below restate the kmer
distance of SURVEY §8a a1/a2 on the GPU path. A GPU Measurer keeps its
genome packed in HBM; `getDistances` is the batched form the processor
should call (GenomePairList.prepare groups pairs by id1, MethodTableProcessor.java:240).
"""
from __future__ import annotations

import threading
from typing import Sequence

from . import _lib as L
from .kmers import Context, KmerSets, KmerType
from .processors import Genome, ParseFailureException


class Measurer:
    def __init__(self, method: "DistanceMethod", genome: Genome):
        self.method = method
        self.genome = genome
        self.sets = KmerSets.from_sequences([method.kmer_text(genome)], method.k, method.kmer_type,
                                            method.flags, method.ctx)


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
        self._lock = threading.Lock()

    def parseParmString(self, parms: str) -> None:
        raise NotImplementedError

    def getMeasurer(self, genome: Genome) -> Measurer:
        return Measurer(self, genome)

    def getDistance(self, measurer: Measurer, genome: Genome) -> float:
        return self.getDistances(measurer, [genome])[0]

    def getDistances(self, measurer: Measurer, genomes: Sequence[Genome]) -> list[float]:
        """Batched getDistance: one device row query for all genomes of an id1 group."""
        with self._lock:
            others = KmerSets.from_sequences([self.kmer_text(g) for g in genomes], self.k, self.kmer_type,
                                             self.flags, self.ctx)
            both = measurer.sets.concat(others)
            d = both.row_query(0, range(1, 1 + len(genomes)), L.QUERY_ALL)
        return [float(x) for x in d]

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
                self.k = int(val)
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
    """Protein kmer distance over a genome's proteins (ProteinKmers, k=8 default)."""
    type_name = "prot"
    kmer_type = KmerType.PROT
    default_k = 8

    def kmer_text(self, g: Genome) -> bytes:
        prots = getattr(g, "proteins", None) or []
        return b"\0".join(p.encode("latin-1") for p in prots)
