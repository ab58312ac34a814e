"""Diagnostic builds (NOT product code; outputs are git-ignored): the sparse
tile kernel's walk with one cost removed at a time, to see where its time
goes. Their counts are WRONG by design; they are only timed, each in a
package copy of its own (scripts/r05/build/diag_<v>/gdist, whose
libgdist.so carries the hash of its own modified sources). Variants:
  d1  counter adds to conflict-free LDS addresses (atomics kept)
  d2  no counter adds (operands still computed)
  d3  the walk's record loads confined to the first 16 KiB of each chunk's
      records (cache hits instead of gathers)
  d4  d2 + d3
  d5  no walk at all (each batch's setup only: list bounds, prefix sums, records)
  d6  d5 without the counters' zeroing and the chunk partial's store
  d7  no batches at all (the chunk's workgroup: zeroing, barriers, partial store)
  d8  the trailing rare-row workgroups return at once
  d9  d7 + d8
Usage: python scripts/r05/diag_build.py d1 d2 ...
"""
import os, shutil, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "genome.distance_amd")
OUT = os.path.join(ROOT, "scripts", "r05", "build")

CNT_ADD = """__device__ __forceinline__ void cnt_add(uint32_t* cnt, uint32_t r, uint32_t c, uint32_t v) {
    atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(cnt) + (r ^ (c >> 16))), v << (c & 31));
}"""
D1 = """__device__ __forceinline__ void cnt_add(uint32_t* cnt, uint32_t r, uint32_t c, uint32_t v) {
    atomicAdd(cnt + (((r ^ (c >> 16)) >> 2) & 0x1FC0u) + (threadIdx.x & 63), v << (c & 31));
}"""
D2 = """__device__ __forceinline__ void cnt_add(uint32_t* cnt, uint32_t r, uint32_t c, uint32_t v) {
    if ((r ^ (c >> 16) ^ v) == 0x7FFFFFF3u) atomicAdd(cnt, v << (c & 31));
}"""
RI22 = "        ci[u] = (uint32_t)r[u].z + ((uint32_t)yc2 << 4);\n    }\n    uint4 a0[SU];"
RI22_D3 = ("        ci[u] = (uint32_t)r[u].z + ((uint32_t)yc2 << 4);\n        ri[u] &= 0x3FF0u; ci[u] &= 0x3FF0u;\n"
           "    }\n    uint4 a0[SU];")
WALK = "    if (MT == 2 && diag && d22) sparse_walk<2, 3>"
WALK_D5 = "    if (total != 0x7FFFFFF3) return;\n    if (MT == 2 && diag && d22) sparse_walk<2, 3>"
ZERO = "    for (int t = threadIdx.x; t < SB * SB / 2; t += SNT) cnt[t] = 0;\n    if (threadIdx.x == 0) next_batch"
ZERO_D6 = "    if (threadIdx.x == 0) next_batch"
STORE = "        for (int t = threadIdx.x; t < SB * SB / 2; t += SNT) dst[t] = cnt[t];"
STORE_D6 = "        if (threadIdx.x == 0x7FFF) dst[0] = cnt[0];"
BATCH = "        global_batch<SUN, MT>(tc, s0, we, -1, lane, wrec, masks, cnt);"
BATCH_D7 = "        if (s0 == 0x7FFFFFF3) global_batch<SUN, MT>(tc, s0, we, -1, lane, wrec, masks, cnt);"
RARE = "        rare_slab_row(rs, (int)(blockIdx.x - ntw), r0, c0, c1, upper, cnt);"
RARE_D8 = "        if (r0 == 0x7FFFFFF3) rare_slab_row(rs, (int)(blockIdx.x - ntw), r0, c0, c1, upper, cnt);"
DG22 = "        ne[u] = xc != yc ? ~0u : 0u;\n"
DG22_D3 = "        ne[u] = xc != yc ? ~0u : 0u;\n        ri[u] &= 0x3FF0u; ci[u] &= 0x3FF0u;\n"


def build(v):
    top = f"/tmp/gdist_diag_{v}"
    shutil.rmtree(top, ignore_errors=True)
    tmp = os.path.join(top, "pkg")
    shutil.copytree(PKG, tmp, ignore=shutil.ignore_patterns("build", "*.so", "__pycache__"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    p = os.path.join(tmp, "csrc", "sparse.hip")
    s = open(p).read()
    assert CNT_ADD in s and RI22 in s and DG22 in s
    if v == "d1":
        s = s.replace(CNT_ADD, D1)
    if v in ("d2", "d4"):
        s = s.replace(CNT_ADD, D2)
    if v == "d6":
        assert ZERO in s and STORE in s
        s = s.replace(WALK, WALK_D5).replace(ZERO, ZERO_D6).replace(STORE, STORE_D6)
    if v in ("d7", "d9"):
        assert BATCH in s
        s = s.replace(BATCH, BATCH_D7)
    if v in ("d8", "d9"):
        assert RARE in s
        s = s.replace(RARE, RARE_D8)
    if v == "d5":
        assert WALK in s
        s = s.replace(WALK, WALK_D5)
    if v in ("d3", "d4"):
        s = s.replace(RI22, RI22_D3).replace(DG22, DG22_D3)
    open(p, "w").write(s)
    subprocess.run(["make", "-s", "-j", "8", "-C", tmp], check=True)
    dst = os.path.join(OUT, f"diag_{v}")
    shutil.rmtree(dst, ignore_errors=True)
    shutil.copytree(os.path.join(tmp, "gdist"), os.path.join(dst, "gdist"),
                    ignore=shutil.ignore_patterns("__pycache__"))
    print("built", v, "->", dst)


for v in sys.argv[1:]:
    build(v)
