"""ctypes binding of libgdist.so (the C-ABI declared in include/gdist.h).

The product path: every call goes to the HIP library. If libgdist.so is
missing this module raises at import time — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgdist.so")

OK, EINVAL, ENOMEM, EDEVICE, ECOMM = 0, -1, -2, -3, -4
DNA, PROT, SKETCH = 0, 1, 2
STRAND_BOTH, STRAND_FWD, STRAND_CANON = 0x0, 0x1, 0x2
AMBIG_DEFAULT, AMBIG_SKIP, AMBIG_KEEP = 0x0, 0x4, 0x8
NO_CASE_FOLD = 0x10
UPPER_TRIANGLE, OUT_DEVICE, EMPTY_NAN, SKETCH_JACCARD = 0x100, 0x200, 0x400, 0x800
METHOD_AUTO, METHOD_SORTED, METHOD_BITSET = 0, 1, 2
BITSET_KEEP_SINGLETONS = 0x1
ALLGATHER_CONSUME = 0x1
QUERY_ALL, QUERY_ANY_LE, QUERY_ARGMIN = 0, 1, 2
UNIQUE_ID_BYTES = 128
OPTION_DEFAULT = -(1 << 63)   # GDIST_OPTION_DEFAULT


class GdistError(RuntimeError):
    """Device / communicator failure (IllegalStateException in the JNI shim)."""


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libgdist.so not found at {LIB_PATH}: build it with "
            "`make -C genome.distance_amd` (or __graft_entry__.build()); "
            "there is no CPU fallback")
    return C.CDLL(LIB_PATH)


lib = _load()

_PKG = os.path.dirname(_HERE)
_REPO = os.path.dirname(_PKG)


def tree_source_hash() -> str:
    """sha256 prefix of the library's sources in this tree, in the Makefile's
    order (csrc/*.hip by name, csrc/gdist_internal.hpp, include/gdist.h)."""
    import glob
    import hashlib
    files = sorted(glob.glob(os.path.join(_PKG, "csrc", "*.hip")))
    files += [os.path.join(_PKG, "csrc", "gdist_internal.hpp"), os.path.join(_REPO, "include", "gdist.h")]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def check_build() -> str:
    """Raises when the loaded libgdist.so was built from other sources than
    this tree's (a stale in-tree build); returns the hash."""
    built = lib.gdist_source_hash().decode()
    tree = tree_source_hash()
    if built != tree:
        raise ImportError(f"libgdist.so is stale: built from sources {built}, this tree is {tree}; "
                          "rebuild with `make -C genome.distance_amd`")
    return built

_i64, _i32, _u32, _dbl = C.c_int64, C.c_int32, C.c_uint, C.c_double
_vp, _i64p, _i32p, _u64p, _dblp = (C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_double))
_ctxp, _setp = C.c_void_p, C.c_void_p

_SIGS = {
    "gdist_version": (C.c_char_p, []),
    "gdist_source_hash": (C.c_char_p, []),
    "gdist_abi_version": (C.c_int, []),
    "gdist_last_error": (C.c_char_p, []),
    "gdist_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "gdist_ctx_create": (C.c_int, [C.c_int, C.POINTER(_ctxp)]),
    "gdist_ctx_destroy": (C.c_int, [_ctxp]),
    "gdist_ctx_synchronize": (C.c_int, [_ctxp]),
    "gdist_ctx_last_timing": (C.c_int, [_ctxp, _dblp, _dblp, _i64p]),
    "gdist_ctx_recent_timings": (C.c_int, [_ctxp, C.c_int, _dblp, C.POINTER(C.c_int)]),
    "gdist_ctx_kernel_ms": (C.c_int, [_ctxp, C.c_int, _dblp]),
    "gdist_ctx_set_option": (C.c_int, [_ctxp, C.c_char_p, _i64]),
    "gdist_ctx_get_option": (C.c_int, [_ctxp, C.c_char_p, _i64p, C.POINTER(C.c_int)]),
    "gdist_ctx_option_name": (C.c_int, [C.c_int, C.POINTER(C.c_char_p)]),
    "gdist_dev_alloc": (C.c_int, [_ctxp, _i64, C.POINTER(_vp)]),
    "gdist_dev_free": (C.c_int, [_ctxp, _vp]),
    "gdist_memcpy_d2h": (C.c_int, [_ctxp, _vp, _vp, _i64]),
    "gdist_memcpy_h2d": (C.c_int, [_ctxp, _vp, _vp, _i64]),
    "gdist_host_alloc": (C.c_int, [_i64, C.POINTER(C.c_void_p)]),
    "gdist_host_free": (C.c_int, [_vp]),
    "gdist_release_cache": (C.c_int, [C.c_int]),
    "gdist_sets_pack": (C.c_int, [_ctxp, C.c_int, C.c_int, _u32, C.c_char_p, _i64p, _i64, C.POINTER(_setp)]),
    "gdist_sets_pack_device": (C.c_int, [_ctxp, C.c_int, C.c_int, _u32, _vp, _vp, _i64, _i64,
                                         C.POINTER(_setp)]),
    "gdist_sets_append": (C.c_int, [_ctxp, _setp, C.c_char_p, _i64p, _i64, _i64p]),
    "gdist_sets_upload": (C.c_int, [_ctxp, C.c_int, C.c_int, _i64, _i64p, _u64p, C.POINTER(_setp)]),
    "gdist_sets_free": (C.c_int, [_setp]),
    "gdist_sets_info": (C.c_int, [_setp, C.POINTER(C.c_int), C.POINTER(C.c_int), _i64p, _i64p]),
    "gdist_sets_sizes": (C.c_int, [_setp, _i64p]),
    "gdist_sets_download": (C.c_int, [_setp, _i64p, _u64p]),
    "gdist_sets_build_bitsets": (C.c_int, [_setp, _u32]),
    "gdist_sets_build_bitsets_ex": (C.c_int, [_setp, _u32, _i64]),
    "gdist_sets_release_codes": (C.c_int, [_setp]),
    "gdist_sets_build_timing": (C.c_int, [_setp, _dblp, _dblp, _dblp, C.POINTER(C.c_int)]),
    "gdist_sets_rare_info": (C.c_int, [_setp, _i64p, _i64p, _i64p]),
    "gdist_sets_rare_stats": (C.c_int, [_setp, _i64p, _i64p]),
    "gdist_sets_rare_kmers": (C.c_int, [_setp, _i64p]),
    "gdist_sets_sparse_info": (C.c_int, [_setp, _i64p, _i64p, _i64p]),
    "gdist_sets_variant_info": (C.c_int, [_setp, _i64p, _i64p, _i64p, _dblp]),
    "gdist_sets_variant_layout": (C.c_int, [_setp, C.POINTER(C.c_int), C.POINTER(C.c_int), _i64p]),
    "gdist_sets_group_info": (C.c_int, [_setp, _i64p, _i64p]),
    "gdist_sets_sparse_sides": (C.c_int, [_setp, _i64p, _i64p]),
    "gdist_sets_sparse_pairs": (C.c_int, [_setp, C.POINTER(C.c_double)]),
    "gdist_sets_bitset_info": (C.c_int, [_setp, _i64p, _i64p]),
    "gdist_sets_bitset_download": (C.c_int, [_setp, _u64p]),
    "gdist_sets_concat": (C.c_int, [_setp, _setp, C.POINTER(_setp)]),
    "gdist_sets_prepare": (C.c_int, [_ctxp, _setp, C.c_int, _dbl, C.POINTER(C.c_int), _dblp, _dblp]),
    "gdist_intersect_matrix": (C.c_int, [_ctxp, _setp, _i64, _i64, _i64, _i64, C.c_int, _u32, _vp, _vp, _i64]),
    "gdist_greedy_reps": (C.c_int, [_ctxp, _setp, C.c_int, _dbl, _i64p, _i32p, _i64p, _dblp, _i64p]),
    "gdist_row_query": (C.c_int, [_ctxp, _setp, _i64, _i64p, _i64, C.c_int, _dbl, _dblp, _i32p, _i64p, _dblp]),
    "gdist_sketch_build": (C.c_int, [_ctxp, _setp, C.c_int, C.POINTER(_setp)]),
    "gdist_sketch_upload": (C.c_int, [_ctxp, C.c_int, _i64, _i64p, _i32p, C.POINTER(_setp)]),
    "gdist_sketch_download": (C.c_int, [_setp, _i64p, _i32p]),
    "gdist_sketch_matrix": (C.c_int, [_ctxp, _setp, _i64, _i64, _i64, _i64, _u32, _vp, _vp, _i64]),
    "gdist_lsh_build": (C.c_int, [_ctxp, _setp, C.c_int, C.c_int, C.c_uint64, C.POINTER(C.c_void_p)]),
    "gdist_lsh_free": (C.c_int, [C.c_void_p]),
    "gdist_lsh_closest": (C.c_int, [_ctxp, C.c_void_p, _setp, C.c_int, _dbl, _i64p, _dblp, _i32p]),
    "gdist_comm_unique_id": (C.c_int, [C.c_char_p]),
    "gdist_comm_init": (C.c_int, [_ctxp, C.c_char_p, C.c_int, C.c_int]),
    "gdist_comm_init_host": (C.c_int, [_ctxp, C.c_int, C.c_int, C.c_void_p, _vp]),
    "gdist_comm_destroy": (C.c_int, [_ctxp]),
    "gdist_sets_allgather": (C.c_int, [_ctxp, _setp, C.POINTER(_setp)]),
    "gdist_sets_allgather_ex": (C.c_int, [_ctxp, _setp, _u32, C.POINTER(_setp)]),
    "gdist_sets_exchange_plan": (C.c_int, [_ctxp, _setp, C.c_int, C.POINTER(C.c_int), _dblp, _dblp]),
    "gdist_sets_allgather_bitsets": (C.c_int, [_ctxp, _setp, _u32, C.POINTER(_setp)]),
    "gdist_comm_allreduce_max": (C.c_int, [_ctxp, _dblp]),
    "gdist_sets_block_cost": (C.c_int, [_setp, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int,
                                        C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "gdist_triangle_partition": (C.c_int, [_i64, C.c_int, _i64, _i64p]),
}

for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_SIGS)

# int (*gdist_allgather_fn)(const void* send, void* recv, int64_t bytes, void* user)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)


def check(rc: int) -> None:
    """Map a status code to the exception the reference throws for it."""
    if rc == OK:
        return
    msg = lib.gdist_last_error().decode(errors="replace")
    if rc == EINVAL:
        raise ValueError(msg)          # IllegalArgumentException / ParseFailureException
    if rc == ENOMEM:
        raise MemoryError(msg)         # OutOfMemoryError
    raise GdistError(f"[{rc}] {msg}")  # IllegalStateException


def ptr(a: np.ndarray, t):
    return a.ctypes.data_as(C.POINTER(t))


def vptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, int):
        return a
    return a.ctypes.data
