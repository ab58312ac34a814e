"""Host-side mirror of the reference's kmer-set API over libgdist.so.

Reference surface (org.theseed:sequence, un-vendored; call sites in-repo):
  KmerType.DNA / KmerType.PROT, getKmerSize(), createKmers(seq, K)
      FastaDistanceProcessor.java:81-96,153,184
  SequenceKmers.distance(other), size(), hashSet(width)
      FastaDistanceProcessor.java:186, SketchProcessor.java:88, WidthProcessor.java:178
  Sketch(int[] signature, name).distance(other), getSignature()
      WidthProcessor.java:178-185
The GPU-native form of these is a *collection*: `KmerSets` holds many kmer
sets packed on the device and answers whole matrices / row queries in one
call; `SequenceKmers` is a per-set view whose `distance()` is kept for API
parity (one pair per call is a correctness path, not a fast path).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import enum
import os
import weakref
from typing import Iterable, Mapping, Sequence

import numpy as np

from . import _lib as L


def option_names() -> list[str]:
    """Every tuning option of gdist_ctx_set_option (include/gdist.h)."""
    names, i = [], 0
    while True:
        p = C.c_char_p()
        if L.lib.gdist_ctx_option_name(i, C.byref(p)) != L.OK:
            return names
        names.append(p.value.decode())
        i += 1


def options_from_env(environ: Mapping[str, str] | None = None) -> dict[str, int]:
    """GDIST_<NAME>=<int> variables of a host program's environment as an
    options dict. The library itself never reads the environment; A/B
    launchers (bench.py, scripts/) map it explicitly with this."""
    env = os.environ if environ is None else environ
    out = {}
    for name in option_names():
        v = env.get("GDIST_" + name.upper())
        if v is not None and v != "":
            out[name] = int(v)
    return out


class Context:
    """One HIP device + stream (gdist_ctx) and its tuning options."""

    _defaults: dict[int, "Context"] = {}

    def __init__(self, device: int = 0, options: Mapping[str, int] | None = None):
        h = C.c_void_p()
        L.check(L.lib.gdist_ctx_create(device, C.byref(h)))
        self.h = h
        self.device = device
        self._handles = weakref.WeakSet()     # live collections: freed before the context
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def set_option(self, name: str, value: int | None) -> None:
        """gdist_ctx_set_option; None restores the default."""
        L.check(L.lib.gdist_ctx_set_option(self.h, name.encode(), L.OPTION_DEFAULT if value is None else int(value)))

    def option(self, name: str) -> int | None:
        """The option's value, None when it is at its default."""
        v, is_set = C.c_int64(), C.c_int()
        L.check(L.lib.gdist_ctx_get_option(self.h, name.encode(), C.byref(v), C.byref(is_set)))
        return int(v.value) if is_set.value else None

    @contextlib.contextmanager
    def options(self, **opts: int | None):
        """Set options for the duration of a with-block, then restore them."""
        old = {k: self.option(k) for k in opts}
        try:
            for k, v in opts.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_option(k, v)

    @classmethod
    def default(cls, device: int = 0) -> "Context":
        if device not in cls._defaults:
            cls._defaults[device] = cls(device)
        return cls._defaults[device]

    def close(self):
        """gdist_ctx_destroy, after freeing every collection still alive on it
        (a collection must not outlive its context)."""
        if self.h:
            for hd in list(self._handles):
                hd.free()
            L.lib.gdist_ctx_destroy(self.h)
            self.h = None

    def synchronize(self):
        L.check(L.lib.gdist_ctx_synchronize(self.h))

    def last_timing(self) -> tuple[float, float, int]:
        k, c, n = C.c_double(), C.c_double(), C.c_int64()
        L.check(L.lib.gdist_ctx_last_timing(self.h, C.byref(k), C.byref(c), C.byref(n)))
        return k.value, c.value, n.value

    KERNEL_FAMILIES = {"sparse": 0, "rare": 1, "dense": 2, "sorted": 3, "variant": 4}

    def kernel_ms(self, family: str) -> float:
        """HIP-event ms of one kernel family's launches (sparse / rare / dense /
        sorted) in the last call made with option time_kernels = 1 (-1: that
        family was not timed)."""
        v = C.c_double()
        L.check(L.lib.gdist_ctx_kernel_ms(self.h, self.KERNEL_FAMILIES[family], C.byref(v)))
        return v.value

    def recent_timings(self, n: int) -> list[float]:
        """Kernel ms of the last n matrix calls, oldest first (waits for them)."""
        out = np.zeros(max(n, 1), dtype=np.float64)
        cnt = C.c_int()
        L.check(L.lib.gdist_ctx_recent_timings(self.h, int(n), L.ptr(out, C.c_double), C.byref(cnt)))
        return [float(x) for x in out[:cnt.value]]

    def alloc(self, nbytes: int) -> "DeviceBuffer":
        return DeviceBuffer(self, nbytes)

    # ---- RCCL communicator (row-sharded multi-GPU)
    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(L.UNIQUE_ID_BYTES)
        L.check(L.lib.gdist_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, uid: bytes, nranks: int, rank: int) -> None:
        L.check(L.lib.gdist_comm_init(self.h, uid, nranks, rank))

    def comm_init_host(self, nranks: int, rank: int, allgather) -> None:
        """Host-staged transport (gdist_comm_init_host): `allgather(np.uint8
        array of n bytes) -> np.uint8 array of nranks * n bytes in rank order`,
        e.g. torch.distributed.all_gather over gloo. For ranks sharing one GPU
        (RCCL refuses that) and tests; RCCL is the multi-GPU transport."""
        def cb(send, recv, nbytes, _user):
            try:
                src = np.ctypeslib.as_array((C.c_uint8 * max(int(nbytes), 1)).from_address(send))[:nbytes]
                out = np.ascontiguousarray(allgather(src.copy()), dtype=np.uint8)
                if out.nbytes != nbytes * nranks:
                    return 1
                if out.nbytes:
                    C.memmove(recv, out.ctypes.data, out.nbytes)
                return 0
            except Exception:
                return 1
        self._host_ag = L.ALLGATHER_FN(cb)          # keep the thunk alive
        L.check(L.lib.gdist_comm_init_host(self.h, nranks, rank, C.cast(self._host_ag, C.c_void_p), None))

    def comm_destroy(self) -> None:
        L.check(L.lib.gdist_comm_destroy(self.h))
        self._host_ag = None

    def allreduce_max(self, v: float) -> float:
        x = C.c_double(v)
        L.check(L.lib.gdist_comm_allreduce_max(self.h, C.byref(x)))
        return x.value


def release_device_cache(device: int = 0) -> None:
    """gdist_release_cache: hand the library's cached device blocks back to
    the driver (before another process takes the GPU)."""
    L.check(L.lib.gdist_release_cache(int(device)))


class HostBuffer:
    """Page-locked host memory (gdist_host_alloc) for sequence bytes: fill
    `array` (uint8) in place, e.g. with a FASTA reader, and pass it to
    KmerSets.from_blob: the pack uploads it with one DMA per chunk instead of
    the runtime's staged pageable copies. `array` must not be used after
    free() / the with-block."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        L.check(L.lib.gdist_host_alloc(int(nbytes), C.byref(p)))
        self.ptr, self.nbytes = p.value or 0, int(nbytes)
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(1, self.nbytes)).from_address(self.ptr))[:self.nbytes]

    def free(self):
        if self.ptr:
            self.array = None
            L.check(L.lib.gdist_host_free(self.ptr))
            self.ptr = 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceBuffer:
    def __init__(self, ctx: Context, nbytes: int):
        p = C.c_void_p()
        L.check(L.lib.gdist_dev_alloc(ctx.h, int(nbytes), C.byref(p)))
        self.ctx, self.ptr, self.nbytes = ctx, p.value or 0, int(nbytes)
        ctx._handles.add(self)

    def to_host(self, dtype, count: int | None = None, offset: int = 0) -> np.ndarray:
        """`count` elements of `dtype` starting at element `offset`."""
        dt = np.dtype(dtype)
        n = (self.nbytes // dt.itemsize - offset) if count is None else count
        if offset < 0 or n < 0 or (offset + n) * dt.itemsize > self.nbytes:
            raise ValueError("read outside the device buffer")
        out = np.empty(n, dtype=dt)
        L.check(L.lib.gdist_memcpy_d2h(self.ctx.h, out.ctypes.data, self.ptr + offset * dt.itemsize,
                                       n * dt.itemsize))
        return out

    def from_host(self, a: np.ndarray, offset: int = 0):
        """Copy `a` into the buffer from element `offset` (in a's dtype) on."""
        a = np.ascontiguousarray(a)
        at = int(offset) * a.itemsize
        if offset < 0 or at + a.nbytes > self.nbytes:
            raise ValueError("write outside the device buffer")
        L.check(L.lib.gdist_memcpy_h2d(self.ctx.h, self.ptr + at, a.ctypes.data, a.nbytes))

    def free(self):
        if self.ptr:
            L.check(L.lib.gdist_dev_free(self.ctx.h, self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class KmerType(enum.Enum):
    """KmerType.DNA / KmerType.PROT (FastaDistanceProcessor.java:81-96)."""
    DNA = (L.DNA, 21)
    PROT = (L.PROT, 8)

    @property
    def kind(self) -> int:
        return self.value[0]

    def getKmerSize(self) -> int:
        return self.value[1]

    def createKmers(self, seq: str | bytes, k: int, flags: int = 0, ctx: Context | None = None) -> "SequenceKmers":
        return KmerSets.from_sequences([seq], k, self, flags, ctx)[0]

    @classmethod
    def parse(cls, name: str) -> "KmerType":
        return cls[name.upper()]


def _as_bytes(s) -> bytes:
    return s if isinstance(s, (bytes, bytearray)) else str(s).encode("latin-1")


class _Handle:
    def __init__(self, ctx: Context, h: C.c_void_p):
        self.ctx, self.h = ctx, h
        ctx._handles.add(self)

    def free(self):
        if getattr(self, "h", None):
            L.lib.gdist_sets_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def info(self):
        kind, k, n, t = C.c_int(), C.c_int(), C.c_int64(), C.c_int64()
        L.check(L.lib.gdist_sets_info(self.h, C.byref(kind), C.byref(k), C.byref(n), C.byref(t)))
        return kind.value, k.value, n.value, t.value

    def __len__(self) -> int:
        return self.info()[2]

    def allgather(self, consume: bool = False):
        """Concatenation of every rank's local collection, in rank order
        (one RCCL all-gather of offsets, one in place of codes / signatures).
        consume=True releases this collection's device data once its codes
        are in the gather buffer (GDIST_ALLGATHER_CONSUME): peak memory is
        then (ranks + 1) x the largest shard instead of + 2 shards."""
        h = C.c_void_p()
        L.check(L.lib.gdist_sets_allgather_ex(self.ctx.h, self.h, L.ALLGATHER_CONSUME if consume else 0,
                                              C.byref(h)))
        return type(self)(self.ctx, h)

    def exchange_plan(self, method: int = L.METHOD_AUTO) -> tuple[int, float, float]:
        """(method, bytes_bitsets, bytes_codes): the exchange every rank of the
        communicator takes for a row-sharded N x N (collective call):
        METHOD_BITSET = the dictionary exchange (allgather_bitsets),
        METHOD_SORTED = the code all-gather (allgather) for the sorted join."""
        m = C.c_int()
        bb, bc = C.c_double(), C.c_double()
        L.check(L.lib.gdist_sets_exchange_plan(self.ctx.h, self.h, method, C.byref(m), C.byref(bb), C.byref(bc)))
        return m.value, bb.value, bc.value


class KmerSets(_Handle):
    """A collection of kmer sets (sorted unique uint64 codes) resident in HBM."""

    @classmethod
    def from_sequences(cls, seqs: Sequence, k: int, kmer_type: KmerType = KmerType.DNA, flags: int = 0,
                       ctx: Context | None = None) -> "KmerSets":
        ctx = ctx or Context.default()
        bs = [_as_bytes(s) for s in seqs]
        off = np.zeros(len(bs) + 1, dtype=np.int64)
        if bs:
            off[1:] = np.cumsum([len(b) for b in bs])
        blob = b"".join(bs) or b"\0"
        h = C.c_void_p()
        L.check(L.lib.gdist_sets_pack(ctx.h, kmer_type.kind, int(k), flags, blob, L.ptr(off, C.c_int64),
                                      len(bs), C.byref(h)))
        return cls(ctx, h)

    def append(self, seqs: Sequence) -> int:
        """gdist_sets_append: pack `seqs` with this collection's kmer spec and
        append them as new sets; returns the index of the first one. Every
        derived representation is rebuilt on the next distance call."""
        bs = [_as_bytes(s) for s in seqs]
        off = np.zeros(len(bs) + 1, dtype=np.int64)
        if bs:
            off[1:] = np.cumsum([len(b) for b in bs])
        blob = b"".join(bs) or b"\0"
        first = C.c_int64()
        L.check(L.lib.gdist_sets_append(self.ctx.h, self.h, blob, L.ptr(off, C.c_int64), len(bs), C.byref(first)))
        return first.value

    @classmethod
    def from_blob(cls, blob, offsets, k: int, kmer_type: KmerType = KmerType.DNA, flags: int = 0,
                  ctx: Context | None = None) -> "KmerSets":
        """Sequences already laid out as one byte buffer (bytes / bytearray /
        uint8 array) with int64 offsets (n + 1): passed to gdist_sets_pack as
        they are, no per-sequence copies (FASTA bytes read into memory)."""
        ctx = ctx or Context.default()
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        n = len(off) - 1
        if isinstance(blob, np.ndarray):
            buf = np.ascontiguousarray(blob, dtype=np.uint8)
            ptr = buf.ctypes.data_as(C.c_char_p) if buf.size else b"\0"
        else:
            buf = blob if len(blob) else b"\0"
            ptr = buf if isinstance(buf, bytes) else (C.c_char * len(buf)).from_buffer(buf)
        h = C.c_void_p()
        L.check(L.lib.gdist_sets_pack(ctx.h, kmer_type.kind, int(k), flags, ptr, L.ptr(off, C.c_int64), n,
                                      C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_device(cls, ctx: Context, d_seqs: int, d_off: int, nseqs: int, total_bytes: int, k: int,
                    kmer_type: KmerType = KmerType.DNA, flags: int = 0) -> "KmerSets":
        h = C.c_void_p()
        L.check(L.lib.gdist_sets_pack_device(ctx.h, kmer_type.kind, int(k), flags, d_seqs, d_off, nseqs,
                                             total_bytes, C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_codes(cls, offsets: np.ndarray, codes: np.ndarray, k: int, kmer_type: KmerType = KmerType.DNA,
                   ctx: Context | None = None) -> "KmerSets":
        ctx = ctx or Context.default()
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        cd = np.ascontiguousarray(codes, dtype=np.uint64)
        if cd.size == 0:
            cd = np.zeros(1, dtype=np.uint64)
        h = C.c_void_p()
        L.check(L.lib.gdist_sets_upload(ctx.h, kmer_type.kind, int(k), len(off) - 1, L.ptr(off, C.c_int64),
                                        L.ptr(cd, C.c_uint64), C.byref(h)))
        return cls(ctx, h)

    def sizes(self) -> np.ndarray:
        n = len(self)
        out = np.zeros(n, dtype=np.int64)
        L.check(L.lib.gdist_sets_sizes(self.h, L.ptr(out, C.c_int64)))
        return out

    def download(self) -> tuple[np.ndarray, np.ndarray]:
        _, _, n, t = self.info()
        off = np.zeros(n + 1, dtype=np.int64)
        codes = np.zeros(max(t, 1), dtype=np.uint64)
        L.check(L.lib.gdist_sets_download(self.h, L.ptr(off, C.c_int64), L.ptr(codes, C.c_uint64)))
        return off, codes[:t]

    def build_bitsets(self, keep_singletons: bool = False, rare_threshold: int = -1) -> tuple[int, int]:
        """Dense bitsets (+ rare-kmer posting lists, see include/gdist.h); returns (dense dictionary, W)."""
        L.check(L.lib.gdist_sets_build_bitsets_ex(self.h, L.BITSET_KEEP_SINGLETONS if keep_singletons else 0,
                                                  rare_threshold))
        return self.bitset_info()

    def release_codes(self) -> None:
        """Drop the codes of a collection whose bitsets are built (gdist_sets_release_codes)."""
        L.check(L.lib.gdist_sets_release_codes(self.h))

    def build_timing(self) -> dict:
        """The last bitset build (gdist_sets_build_timing): wall ms, the split stages'
        ms over all shares and of the largest share, the shares, and one rank's
        projected build (wall - split + largest share)."""
        b, sp, mx, n = C.c_double(), C.c_double(), C.c_double(), C.c_int()
        L.check(L.lib.gdist_sets_build_timing(self.h, C.byref(b), C.byref(sp), C.byref(mx), C.byref(n)))
        return {"build_ms": b.value, "split_ms": sp.value, "share_max_ms": mx.value, "shares": n.value,
                "rank_ms": b.value - sp.value + mx.value}

    def prepare(self, method: int = L.METHOD_AUTO, pairs: float = -1.0) -> tuple[int, float, float]:
        """Build the representation `method` needs for `pairs` pairs (-1: the whole
        triangle); returns (method a matrix call will run, bitset cost estimate s
        (-1 without bitsets), sorted cost estimate s). See gdist_sets_prepare."""
        m, cb, cs = C.c_int(), C.c_double(), C.c_double()
        L.check(L.lib.gdist_sets_prepare(self.ctx.h, self.h, method, float(pairs), C.byref(m), C.byref(cb),
                                         C.byref(cs)))
        return m.value, cb.value, cs.value

    def greedy_reps(self, max_dist: float, assign: bool = False, tie_rank: np.ndarray | None = None,
                    method: int = L.METHOD_AUTO):
        """Greedy representatives on the device (gdist_greedy_reps). Returns
        is_rep (int32[N]); with assign=True also (rep_of int64[N], rep_dist
        float64[N]): each set's closest representative, ties to the lowest
        tie_rank (default: index)."""
        n = len(self)
        is_rep = np.zeros(max(n, 1), dtype=np.int32)
        nreps = C.c_int64()
        rep_of = np.zeros(max(n, 1), dtype=np.int64) if assign else None
        rep_d = np.zeros(max(n, 1), dtype=np.float64) if assign else None
        tr = None
        if tie_rank is not None:
            tr = np.ascontiguousarray(tie_rank, dtype=np.int64)
            assert tr.shape == (n,)
        L.check(L.lib.gdist_greedy_reps(self.ctx.h, self.h, method, float(max_dist),
                                        L.ptr(tr, C.c_int64) if tr is not None else None, L.ptr(is_rep, C.c_int32),
                                        L.ptr(rep_of, C.c_int64) if assign else None,
                                        L.ptr(rep_d, C.c_double) if assign else None, C.byref(nreps)))
        if assign:
            return is_rep[:n], rep_of[:n], rep_d[:n]
        return is_rep[:n]

    def block_cost(self, rows: tuple[int, int], cols: tuple[int, int] | None = None,
                   upper: bool = True) -> tuple[float, int]:
        """(modelled seconds, rare kernel: 0 list-major / 1 row-major / -1 none)
        of one matrix call on the block (gdist_sets_block_cost)."""
        c = cols if cols is not None else (0, len(self))
        t, rk = C.c_double(), C.c_int()
        L.check(L.lib.gdist_sets_block_cost(self.h, rows[0], rows[1], c[0], c[1], 1 if upper else 0, C.byref(t),
                                            C.byref(rk)))
        return t.value, rk.value

    def sparse_info(self) -> tuple[int, int, int]:
        """(complement-sparse words, dense words left to the tiles, complement entries)."""
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(L.lib.gdist_sets_sparse_info(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def variant_info(self) -> tuple[int, int, int, float]:
        """(kmers, words, entries, products) of the variant tier (gdist_sets_variant_info)."""
        a, b, c, d = C.c_int64(), C.c_int64(), C.c_int64(), C.c_double()
        L.check(L.lib.gdist_sets_variant_info(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return a.value, b.value, c.value, d.value

    def variant_layout(self) -> tuple[int, int, int]:
        """(kmers a word, bytes a list member, largest row weight) of the
        variant tier (gdist_sets_variant_layout): (16, 4, w) for the grouped
        rare tier of <= 65,536 sets (option rare_group), (47, 8, 0) for C4's
        packed members, (64, 12, 0) unpacked."""
        wk, mb, rw = C.c_int(), C.c_int(), C.c_int64()
        L.check(L.lib.gdist_sets_variant_layout(self.h, C.byref(wk), C.byref(mb), C.byref(rw)))
        return wk.value, mb.value, rw.value

    def group_info(self) -> tuple[int, int]:
        """(groups, grouped sparse words) of the group tier (gdist_sets_group_info)."""
        g, w = C.c_int64(), C.c_int64()
        L.check(L.lib.gdist_sets_group_info(self.h, C.byref(g), C.byref(w)))
        return g.value, w.value

    def sparse_sides(self) -> tuple[int, int]:
        """(complement-sparse words, positive-sparse words)."""
        a, b = C.c_int64(), C.c_int64()
        L.check(L.lib.gdist_sets_sparse_sides(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def sparse_pairs(self) -> float:
        """The sparse tile kernel's products: sum over sparse words of z (z - 1) / 2."""
        p = C.c_double()
        L.check(L.lib.gdist_sets_sparse_pairs(self.h, C.byref(p)))
        return p.value

    def rare_kmers(self) -> int:
        """Rare-tier kmers before identical posting lists were merged."""
        n = C.c_int64()
        L.check(L.lib.gdist_sets_rare_kmers(self.h, C.byref(n)))
        return n.value

    def rare_info(self) -> tuple[int, int, int]:
        """(threshold T, distinct posting lists, their records) of the rare tier."""
        t, n, r = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(L.lib.gdist_sets_rare_info(self.h, C.byref(t), C.byref(n), C.byref(r)))
        return t.value, n.value, r.value

    def rare_stats(self) -> tuple[int, int]:
        """(pair increments, longest posting list) of the rare tier."""
        i, m = C.c_int64(), C.c_int64()
        L.check(L.lib.gdist_sets_rare_stats(self.h, C.byref(i), C.byref(m)))
        return i.value, m.value

    def bitsets(self) -> np.ndarray:
        """The dictionary-rank bitsets, (nsets, W) uint64."""
        n = len(self)
        _, w = self.bitset_info()
        out = np.zeros((n, max(w, 1)), dtype=np.uint64)
        L.check(L.lib.gdist_sets_bitset_download(self.h, L.ptr(out, C.c_uint64)))
        return out[:, :w]

    def bitset_info(self) -> tuple[int, int]:
        d, w = C.c_int64(), C.c_int64()
        L.check(L.lib.gdist_sets_bitset_info(self.h, C.byref(d), C.byref(w)))
        return d.value, w.value

    def allgather_bitsets(self, keep_singletons: bool = False) -> "KmerSets":
        """Bitsets of every rank's sets over one global dictionary (bitset-only collection)."""
        h = C.c_void_p()
        L.check(L.lib.gdist_sets_allgather_bitsets(self.ctx.h, self.h,
                                                   L.BITSET_KEEP_SINGLETONS if keep_singletons else 0,
                                                   C.byref(h)))
        return KmerSets(self.ctx, h)

    def concat(self, other: "KmerSets") -> "KmerSets":
        h = C.c_void_p()
        L.check(L.lib.gdist_sets_concat(self.h, other.h, C.byref(h)))
        return KmerSets(self.ctx, h)

    def matrix(self, rows: tuple[int, int] | None = None, cols: tuple[int, int] | None = None,
               upper: bool = False, method: int = L.METHOD_AUTO, flags: int = 0,
               want_I: bool = True, want_D: bool = True):
        """|A_i ∩ A_j| and distances for rows × cols (host numpy outputs)."""
        n = len(self)
        r0, r1 = rows or (0, n)
        c0, c1 = cols or (0, n)
        nr, nc = r1 - r0, c1 - c0
        I = np.full((nr, nc), -1, dtype=np.int32) if want_I else None
        D = np.full((nr, nc), np.nan, dtype=np.float64) if want_D else None
        fl = flags | (L.UPPER_TRIANGLE if upper else 0)
        L.check(L.lib.gdist_intersect_matrix(self.ctx.h, self.h, r0, r1, c0, c1, method, fl, L.vptr(I),
                                             L.vptr(D), max(nc, 1)))
        return I, D

    def matrix_device(self, d_I: int | None, d_D: int | None, ld: int, rows: tuple[int, int],
                      cols: tuple[int, int], upper: bool = False, method: int = L.METHOD_AUTO,
                      flags: int = 0) -> None:
        fl = flags | L.OUT_DEVICE | (L.UPPER_TRIANGLE if upper else 0)
        L.check(L.lib.gdist_intersect_matrix(self.ctx.h, self.h, rows[0], rows[1], cols[0], cols[1], method,
                                             fl, d_I, d_D, ld))

    def row_query(self, q: int, cols: Iterable[int], mode: int = L.QUERY_ALL, t: float = 1.0):
        cl = np.ascontiguousarray(np.fromiter(cols, dtype=np.int64))
        D = np.zeros(max(len(cl), 1), dtype=np.float64)
        hit, bi, bd = C.c_int32(0), C.c_int64(-1), C.c_double(1.0)
        L.check(L.lib.gdist_row_query(self.ctx.h, self.h, q, L.ptr(cl, C.c_int64) if len(cl) else None,
                                      len(cl), mode, t, L.ptr(D, C.c_double), C.byref(hit), C.byref(bi),
                                      C.byref(bd)))
        if mode == L.QUERY_ANY_LE:
            return bool(hit.value)
        if mode == L.QUERY_ARGMIN:
            return int(bi.value), float(bd.value)
        return D[:len(cl)]

    def sketches(self, width: int) -> "SketchSets":
        h = C.c_void_p()
        L.check(L.lib.gdist_sketch_build(self.ctx.h, self.h, int(width), C.byref(h)))
        return SketchSets(self.ctx, h)

    def __getitem__(self, i: int) -> "SequenceKmers":
        n = len(self)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(i)
        return SequenceKmers(self, i)


class SequenceKmers:
    """SequenceKmers view of one set of a KmerSets collection."""

    def __init__(self, sets: KmerSets, index: int):
        self.sets, self.index = sets, index

    def size(self) -> int:
        return int(self.sets.sizes()[self.index])

    def distance(self, other: "SequenceKmers") -> float:
        """SequenceKmers.distance(other) — FastaDistanceProcessor.java:186."""
        if other.sets is self.sets:
            return float(self.sets.row_query(self.index, [other.index])[0])
        both = self.sets.concat(other.sets)
        return float(both.row_query(self.index, [len(self.sets) + other.index])[0])

    def similarity(self, other: "SequenceKmers") -> int:
        if other.sets is self.sets:
            I, _ = self.sets.matrix((self.index, self.index + 1), (other.index, other.index + 1), want_D=False)
            return int(I[0, 0])
        both = self.sets.concat(other.sets)
        j = len(self.sets) + other.index
        I, _ = both.matrix((self.index, self.index + 1), (j, j + 1), want_D=False)
        return int(I[0, 0])

    def hashSet(self, width: int) -> np.ndarray:
        """SequenceKmers.hashSet(width) — SketchProcessor.java:88."""
        return self.sets.sketches(width).signature(self.index)


class SketchSets(_Handle):
    """Bottom-s MinHash signatures (int32) resident in HBM."""

    @classmethod
    def from_signatures(cls, sigs: Sequence[np.ndarray], width: int, ctx: Context | None = None) -> "SketchSets":
        ctx = ctx or Context.default()
        off = np.zeros(len(sigs) + 1, dtype=np.int64)
        if sigs:
            off[1:] = np.cumsum([len(s) for s in sigs])
        flat = np.concatenate([np.asarray(s, dtype=np.int32) for s in sigs]) if sigs else np.zeros(0, np.int32)
        if flat.size == 0:
            flat = np.zeros(1, dtype=np.int32)
        h = C.c_void_p()
        L.check(L.lib.gdist_sketch_upload(ctx.h, int(width), len(sigs), L.ptr(off, C.c_int64),
                                          L.ptr(np.ascontiguousarray(flat), C.c_int32), C.byref(h)))
        return cls(ctx, h)

    def download(self) -> tuple[np.ndarray, np.ndarray]:
        _, _, n, t = self.info()
        off = np.zeros(n + 1, dtype=np.int64)
        sig = np.zeros(max(t, 1), dtype=np.int32)
        L.check(L.lib.gdist_sketch_download(self.h, L.ptr(off, C.c_int64), L.ptr(sig, C.c_int32)))
        return off, sig[:t]

    def signature(self, i: int) -> np.ndarray:
        off, sig = self.download()
        return sig[off[i]:off[i + 1]].copy()

    def matrix(self, rows=None, cols=None, upper: bool = False, flags: int = 0):
        n = len(self)
        r0, r1 = rows or (0, n)
        c0, c1 = cols or (0, n)
        nr, nc = r1 - r0, c1 - c0
        common = np.full((nr, nc), -1, dtype=np.int32)
        D = np.full((nr, nc), np.nan, dtype=np.float64)
        fl = flags | (L.UPPER_TRIANGLE if upper else 0)
        L.check(L.lib.gdist_sketch_matrix(self.ctx.h, self.h, r0, r1, c0, c1, fl, common.ctypes.data,
                                          D.ctypes.data, max(nc, 1)))
        return common, D

    def matrix_device(self, d_common: int | None, d_D: int | None, ld: int, rows, cols, upper=False, flags=0):
        fl = flags | L.OUT_DEVICE | (L.UPPER_TRIANGLE if upper else 0)
        L.check(L.lib.gdist_sketch_matrix(self.ctx.h, self.h, rows[0], rows[1], cols[0], cols[1], fl, d_common,
                                          d_D, ld))


class LSHIndex:
    """LSHMemSeqHash over a SketchSets collection (gdist_lsh_build):
    getClosest(queries, n, maxDist) per query sketch."""

    def __init__(self, sketches: "SketchSets", stages: int, buckets: int, seed: int = 0x5EED):
        h = C.c_void_p()
        L.check(L.lib.gdist_lsh_build(sketches.ctx.h, sketches.h, int(stages), int(buckets), int(seed), C.byref(h)))
        self.ctx, self.h, self.sketches = sketches.ctx, h, sketches      # the index keeps its sketches alive
        self.ctx._handles.add(self)

    def free(self):
        if getattr(self, "h", None):
            L.lib.gdist_lsh_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def getClosest(self, queries: "SketchSets", n: int, max_dist: float) -> list[list[tuple[int, float]]]:
        """For each query: [(indexed set, distance)] nearest first, at most n, distance <= max_dist."""
        nq = len(queries)
        idx = np.zeros(max(nq * n, 1), dtype=np.int64)
        d = np.zeros(max(nq * n, 1), dtype=np.float64)
        cnt = np.zeros(max(nq, 1), dtype=np.int32)
        L.check(L.lib.gdist_lsh_closest(self.ctx.h, self.h, queries.h, int(n), float(max_dist),
                                        L.ptr(idx, C.c_int64), L.ptr(d, C.c_double), L.ptr(cnt, C.c_int32)))
        return [[(int(idx[q * n + r]), float(d[q * n + r])) for r in range(cnt[q])] for q in range(nq)]


def triangle_partition(n: int, nparts: int, align: int = 1) -> list[int]:
    """Row bounds with equal upper-triangle area per part."""
    b = np.zeros(nparts + 1, dtype=np.int64)
    L.check(L.lib.gdist_triangle_partition(n, nparts, align, L.ptr(b, C.c_int64)))
    return [int(x) for x in b]
