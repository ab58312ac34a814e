"""Synthetic genomes of SURVEY.md §8(d) (no datasets are reachable here).

PRNG: splitmix64, master seed 0x5EED_0000 + cfg, per-genome substream
seed ^ (g * 0x9E3779B97F4A7C15). DNA: an ancestor i.i.d. uniform over ACGT;
genome g is the ancestor with round(p_g * L) substitutions at splitmix
positions, p_g = u_g * p_max. Protein: the same over the 20 standard amino
acids. Fixed lengths (no indels). realistic_genome(): clades, indels and segment
moves over either alphabet (the C2 / C3 / C4 realistic twins).
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
DNA_ALPHA = np.frombuffer(b"ACGT", dtype=np.uint8)
AA_ALPHA = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """n outputs of the splitmix64 stream seeded with `seed` (vectorised)."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _uniform(x: np.ndarray) -> np.ndarray:
    return (x >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def master_seed(cfg: int) -> int:
    return 0x5EED0000 + cfg


def genomes(n: int, length: int, p_max: float, cfg: int, protein: bool = False,
            first: int = 0) -> np.ndarray:
    """Genomes first..first+n-1 as an (n, length) uint8 array of ASCII letters."""
    alpha = AA_ALPHA if protein else DNA_ALPHA
    a = len(alpha)
    seed = master_seed(cfg)
    anc_idx = (splitmix64(seed, length) % np.uint64(a)).astype(np.uint8)
    out = np.empty((n, length), dtype=np.uint8)
    for r in range(n):
        g = first + r
        with np.errstate(over="ignore"):
            sg = int(np.uint64(seed) ^ (np.uint64(g) * GOLDEN))
        head = splitmix64(sg, 1)
        p = float(_uniform(head)[0]) * p_max
        m = int(round(p * length))
        idx = anc_idx.copy()
        if m:
            x = splitmix64(sg, 2 * m, start=1)
            pos = (x[:m] % np.uint64(length)).astype(np.int64)
            shift = (x[m:] % np.uint64(a - 1)).astype(np.uint8) + 1
            idx[pos] = (idx[pos] + shift) % a
        out[r] = alpha[idx]
    return out


def to_blob(arr: np.ndarray) -> tuple[bytes, np.ndarray]:
    """(concatenated bytes, offsets) of an (n, L) genome array."""
    n, length = arr.shape
    off = np.arange(n + 1, dtype=np.int64) * length
    return arr.tobytes(), off


_ANCESTORS: dict = {}
_COMP = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGT", b"TGCA"):
    _COMP[_a] = _b


def realistic_genome(g: int, length: int, p_max: float, cfg: int, clades: int = 8, p_clade: float = 0.004,
                     indel_rate: float = 2e-5, blocks: int = 16, p_rearrange: float = 0.5,
                     protein: bool = False) -> bytes:
    """Genome g of a collection that is NOT one ancestor plus independent
    substitutions (the structure the locus order was tuned on):
      * clades: the ancestor gets p_clade substitutions per clade (genome g
        belongs to clade g mod `clades`), so genomes share variants in groups
        and the first sequences (the guides) are ordinary clade members;
      * substitutions of its own at p_g ~ U[0, p_max];
      * short indels (1-10 symbols, rate indel_rate per site each way), so
        lengths and kmer windows shift;
      * with probability p_rearrange, 1-3 moves of one of `blocks` equal
        segments to another position, DNA reverse-complemented half the time.
    protein=True: the same over the 20 amino acids (a proteome; moved
    segments are not reversed). Deterministic per (cfg, g, kind): splitmix64
    substreams as genomes()."""
    alpha = AA_ALPHA if protein else DNA_ALPHA
    na = len(alpha)
    seed = master_seed(cfg) ^ (0x5EA1 if not protein else 0x5EA2)
    c = g % clades
    with np.errstate(over="ignore"):
        sc = int(np.uint64(seed) ^ (np.uint64(0xC1ADE + c) * GOLDEN))
        sg = int(np.uint64(seed) ^ (np.uint64(g) * GOLDEN))
    key = (seed, length, na)
    if key not in _ANCESTORS:
        _ANCESTORS.clear()
        _ANCESTORS[key] = (splitmix64(seed, length) % np.uint64(na)).astype(np.uint8)
    idx = _ANCESTORS[key].copy()

    def substitute(idx, s, m, start):
        if m <= 0:
            return
        x = splitmix64(s, 2 * m, start=start)
        pos = (x[:m] % np.uint64(len(idx))).astype(np.int64)
        idx[pos] = (idx[pos] + (x[m:] % np.uint64(na - 1)).astype(np.uint8) + 1) % na

    substitute(idx, sc, int(round(p_clade * length)), 1)
    p = float(_uniform(splitmix64(sg, 1))[0]) * p_max
    substitute(idx, sg, int(round(p * length)), 1)
    seq = alpha[idx]
    # indels at distinct sorted positions: even events delete 1-10 bp, odd
    # events insert 1-10 random bp; assembled in one pass
    ne = int(round(indel_rate * length))
    if ne:
        x = splitmix64(sg, 4 * ne, start=1 << 40)
        pos = np.unique((x[:2 * ne] % np.uint64(length)).astype(np.int64))
        lens = (x[2 * ne:2 * ne + len(pos)] % np.uint64(10)).astype(np.int64) + 1
        pieces, at = [], 0
        for k, q in enumerate(pos):
            if q < at:
                continue
            pieces.append(seq[at:q])
            ln = int(lens[k])
            if k % 2 == 0:
                at = q + ln                                   # deletion
            else:
                pieces.append(alpha[(splitmix64(sg ^ 0x1D, ln, start=int(q)) % np.uint64(na)).astype(np.uint8)])
                at = q
        pieces.append(seq[at:])
        seq = np.concatenate(pieces)
    # rearrangements: move (and maybe reverse-complement) whole segments
    r = splitmix64(sg, 8, start=1 << 41)
    if _uniform(r[:1])[0] < p_rearrange:
        segs = np.array_split(seq, blocks)
        for t in range(1 + int(r[1] % np.uint64(3))):
            a = int(r[2 + t] % np.uint64(len(segs)))
            b = int((r[2 + t] >> np.uint64(20)) % np.uint64(len(segs)))
            s = segs.pop(a)
            if not protein and (r[2 + t] >> np.uint64(40)) & np.uint64(1):
                s = _COMP[s[::-1]]
            segs.insert(b, s)
        seq = np.concatenate(segs)
    return seq.tobytes()


def realistic_genomes(n: int, length: int, p_max: float, cfg: int, first: int = 0, **kw) -> list[bytes]:
    return [realistic_genome(first + r, length, p_max, cfg, **kw) for r in range(n)]
