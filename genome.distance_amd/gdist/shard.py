"""Row-block sharding of the N×N upper triangle across ranks.

Rank g of G owns rows [r_g, r_{g+1}) with r_g = N (1 - sqrt(1 - g/G)),
rounded to row tiles, so every rank holds the same triangle area; it needs
every column, which arrive by one all-gather of the packed sets. There is
no data-path reduction: each rank keeps its own row block of results.
This module is the host logic only (partition, per-rank work, merge); it is
pure Python so the multi-rank path is testable on CPU with gloo.
"""
from __future__ import annotations

import math

import numpy as np


def triangle_bounds(n: int, nparts: int, align: int = 1) -> list[int]:
    b = [0]
    for g in range(1, nparts):
        r = n * (1.0 - math.sqrt(1.0 - g / nparts))
        v = int(math.floor(r / align + 0.5)) * align   # llround (half away from zero)
        b.append(min(n, max(b[-1], v)))
    b.append(n)
    return b


def balanced_bounds(n: int, nparts: int, cost) -> list[int]:
    """Row blocks [b[g], b[g+1]) of the upper triangle minimising the largest
    modelled block time cost(r0, r1) (monotone: non-decreasing in r1,
    non-increasing in r0), e.g. KmerSets.block_cost (gdist_sets_block_cost:
    dense tiles by area, the rare kernel each block would pick by its rows and
    pairs). Bisection on the target time; each block takes rows greedily
    while it stays within the target. Exact integer rows; a cost proportional
    to area gives the equal-area partition (up to a row)."""
    if nparts <= 1 or n == 0:
        return [0] + [n] * max(nparts, 1)

    def cut(target: float) -> list[int] | None:
        b = [0]
        for _ in range(nparts - 1):
            r0 = b[-1]
            lo, hi = r0, n                         # largest r1 with cost(r0, r1) <= target
            while lo < hi:
                mid = (lo + hi + 1) // 2
                if cost(r0, mid) <= target:
                    lo = mid
                else:
                    hi = mid - 1
            b.append(lo)
            if lo == n:
                break
        b += [n] * (nparts + 1 - len(b))
        return b if cost(b[-2], n) <= target else None

    lo_t, hi_t = 0.0, cost(0, n)
    best = cut(hi_t)
    for _ in range(48):
        mid = 0.5 * (lo_t + hi_t)
        b = cut(mid)
        if b is None:
            lo_t = mid
        else:
            hi_t, best = mid, b
        if hi_t - lo_t <= 1e-6 * hi_t:
            break
    return best


def shard_of_sets(n: int, nparts: int) -> list[tuple[int, int]]:
    """Contiguous equal shards of set indices (who packs which genomes)."""
    q, r = divmod(n, nparts)
    out, at = [], 0
    for g in range(nparts):
        m = q + (1 if g < r else 0)
        out.append((at, at + m))
        at += m
    return out


def pairs_in_rows(n: int, r0: int, r1: int) -> int:
    """Upper-triangle pairs (i < j) with r0 <= i < r1."""
    return sum(n - 1 - i for i in range(r0, r1)) if r1 > r0 else 0


def merge_row_blocks(blocks: list[tuple[int, int, np.ndarray]], n: int) -> np.ndarray:
    """Assemble (r0, r1, D_block) pieces into an n×n upper triangle (NaN elsewhere)."""
    D = np.full((n, n), np.nan)
    for r0, r1, blk in blocks:
        for a in range(r0, r1):
            D[a, a + 1:] = blk[a - r0, a + 1:]
    return D
