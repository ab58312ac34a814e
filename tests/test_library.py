"""CPU: libgdist.so loads and exports every symbol include/gdist.h declares;
host-only entry points behave; no compute call is made without a GPU."""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gdist.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gdist_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from gdist import _lib
    syms = declared_symbols()
    assert len(syms) >= 30
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.EXPORTED), "Python binding out of sync with include/gdist.h"


def test_library_built_from_this_tree():
    """The in-tree libgdist.so was built from these sources (the Makefile's
    compiled-in hash vs the tree's): a stale binary fails here, on the CPU
    and on the GPU box alike (test_gpu_options repeats it there)."""
    from gdist import _lib
    assert _lib.check_build() == _lib.tree_source_hash()


def test_abi_version_and_errors():
    from gdist import _lib
    assert _lib.lib.gdist_abi_version() == 1
    assert b"gfx950" in _lib.lib.gdist_version()
    b = np.zeros(5, dtype=np.int64)
    assert _lib.lib.gdist_triangle_partition(-1, 4, 1, _lib.ptr(b, ctypes.c_int64)) == _lib.EINVAL
    assert b"bad partition" in _lib.lib.gdist_last_error()


def test_triangle_partition_matches_host_logic():
    from gdist import kmers, shard
    for n in (0, 1, 10, 1000, 100000):
        for g in (1, 2, 3, 4, 8):
            for align in (1, 64, 128):
                assert kmers.triangle_partition(n, g, align) == shard.triangle_bounds(n, g, align)


def test_triangle_partition_balances_area():
    from gdist import shard
    n = 100000
    b = shard.triangle_bounds(n, 8, 128)
    areas = [shard.pairs_in_rows(n, b[g], b[g + 1]) for g in range(8)]
    assert sum(areas) == n * (n - 1) // 2
    assert max(areas) / min(areas) < 1.05   # 128-row alignment moves ≤ 128·N pairs per boundary


def test_package_import_has_no_cpu_fallback():
    import gdist
    assert gdist._lib.lib is not None
    src = open(os.path.join(ROOT, "genome.distance_amd", "gdist", "kmers.py")).read()
    assert "oracle" not in src and "pyref" not in src
