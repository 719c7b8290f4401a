"""Batch sharding across GPUs: contiguous ranges, each a
multiple of 512 items so every shard starts on a bitmap byte and on a 64-lane
wave boundary.  The shards are independent -- no collective; the per-shard
bitmaps are concatenated.  Mirrors plan_shards() in csrc/pbftv_api.cpp, which
does the same split across the devices of one context."""
from __future__ import annotations

import numpy as np

SHARD_ALIGN = 512


def plan_shards(n: int, parts: int, align: int = SHARD_ALIGN) -> list[tuple[int, int]]:
    if n <= 0:
        return []
    per = -(-n // parts)
    per = -(-per // align) * align
    return [(lo, min(n, lo + per)) for lo in range(0, n, per)]


def shard_of(n: int, parts: int, index: int, align: int = SHARD_ALIGN) -> tuple[int, int]:
    sh = plan_shards(n, parts, align)
    return sh[index] if index < len(sh) else (n, n)


def concat_bitmaps(n: int, shards: list[tuple[int, int]], bitmaps: list[np.ndarray]) -> np.ndarray:
    """Place each shard's LSB-first bitmap at byte offset lo/8 of the global bitmap."""
    out = np.zeros((n + 7) // 8, np.uint8)
    for (lo, hi), bm in zip(shards, bitmaps):
        assert lo % 8 == 0
        nb = (hi - lo + 7) // 8
        out[lo // 8:lo // 8 + nb] = bm[:nb]
    return out
