"""Synthetic genomes of SURVEY.md §8(d) (no datasets are reachable here).

PRNG: splitmix64, master seed 0x5EED_0000 + cfg, per-genome substream
seed ^ (g * 0x9E3779B97F4A7C15). DNA: an ancestor i.i.d. uniform over ACGT;
genome g is the ancestor with round(p_g * L) substitutions at splitmix
positions, p_g = u_g * p_max. Protein: the same over the 20 standard amino
acids. Fixed lengths (no indels).
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
