"""gdist — MI355X-native pairwise kmer-distance hot path of SEEDtk genome.distance.

Python host mirror of the reference API over the C-ABI library libgdist.so
(include/gdist.h). Importing this package loads the HIP library and fails
loudly if it is missing: there is no CPU fallback on the product path.
"""
from . import _lib
from ._lib import (AMBIG_DEFAULT, AMBIG_KEEP, AMBIG_SKIP, BITSET_KEEP_SINGLETONS, EMPTY_NAN, METHOD_AUTO,
                   METHOD_BITSET, METHOD_SORTED, NO_CASE_FOLD, QUERY_ALL, QUERY_ANY_LE, QUERY_ARGMIN,
                   SKETCH_JACCARD, STRAND_BOTH, STRAND_CANON, STRAND_FWD, UPPER_TRIANGLE, GdistError)
from .fasta import Sequence, read_fasta, write_fasta
from .javafmt import java_double, java_doubles
from .kmers import (Context, DeviceBuffer, HostBuffer, release_device_cache, KmerSets, KmerType, LSHIndex, SequenceKmers, SketchSets, option_names,
                    options_from_env, triangle_partition)

__version__ = _lib.lib.gdist_version().decode()


def device_count() -> int:
    import ctypes as C
    n = C.c_int(0)
    _lib.check(_lib.lib.gdist_device_count(C.byref(n)))
    return n.value
