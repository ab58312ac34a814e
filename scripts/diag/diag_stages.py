import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "genome.distance_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import gdist, oracle
from gdist import synth, _lib as L
ctx = gdist.Context.default(0)
seqs = [bytes(r) for r in synth.genomes(300, 3000, 0.05, 91)]
s2 = [bytes(r) for r in synth.genomes(150, 5000, 0.01, 92)]
off, codes = oracle.pack(s2, 21)
blob = b"".join(s2); so = np.zeros(151, np.int64); so[1:] = np.cumsum([len(x) for x in s2])
# host expectation of the extract stage: window order, fwd & rc per window
n = 150 * (5000 - 21 + 1) * 2
f = L.lib.gdist_debug_pack_stages
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint, C.c_char_p, C.POINTER(C.c_int64), C.c_int64] + [C.c_void_p] * 6 + [C.POINTER(C.c_void_p)]
def work():
    for method in ["sorted", "bitset"]:
        sets = gdist.KmerSets.from_sequences(seqs, 15, gdist.KmerType.DNA, 0, ctx)
        if method != "sorted": sets.build_bitsets()
        sets.matrix(method=gdist.METHOD_SORTED if method == "sorted" else gdist.METHOD_BITSET)
        del sets
ref = None
for trial in range(10):
    work()
    bufs = [np.zeros(n, np.uint64), np.zeros(n, np.int32), np.zeros(n, np.uint64), np.zeros(n, np.int32),
            np.zeros(n, np.uint64), np.zeros(n, np.int32)]
    h = C.c_void_p()
    rc = f(ctx.h, 0, 21, 0, blob, so.ctypes.data_as(C.POINTER(C.c_int64)), 150, *[b.ctypes.data for b in bufs], C.byref(h))
    assert rc == 0, L.lib.gdist_last_error()
    sets = gdist.KmerSets(ctx, h)
    o2, c2 = sets.download()
    ok = np.array_equal(c2, codes)
    ke, ve, k1, v1, k2, v2 = bufs
    # independent checks per stage
    e1 = np.sort(ke, kind="stable"); 
    s1_ok = np.array_equal(k1, np.sort(ke)) and np.array_equal(np.sort(v1), np.sort(ve))
    order = np.lexsort((ke, ve))
    s2_ok = np.array_equal(k2, ke[order]) and np.array_equal(v2, ve[order])
    if ref is None and ok:
        ref = [b.copy() for b in bufs]
    ext_ok = ref is None or (np.array_equal(ke, ref[0]) and np.array_equal(ve, ref[1]))
    print(f"trial {trial}: final ok={ok} extract_same_as_good={ext_ok} sort1_ok={s1_ok} sort2_ok={s2_ok}", flush=True)
    del sets
