"""Data-parallel partitioning helpers: contiguous row ranges per rank
(rank order = global row order, which is what the gathered actions and the CSV byte-range
sharding assume) and 64-row-aligned chunking for streamed ingest into the fragment layouts."""
from __future__ import annotations

from typing import Iterator, Tuple

__all__ = ["row_range", "shard_rows", "aligned_chunks", "shard_byte_range"]


def row_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """[lo, hi) of ``rank``'s contiguous share of ``n`` rows (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return n * rank // world, n * (rank + 1) // world


def shard_rows(t, rank: int, world: int, dim: int = -1):
    """This rank's slice of a tensor along its row dimension (feature-major ``[d, n]``: dim -1)."""
    n = t.shape[dim]
    lo, hi = row_range(n, rank, world)
    return t.narrow(dim, lo, hi - lo)


def aligned_chunks(n: int, chunk_rows: int, align: int = 64) -> Iterator[Tuple[int, int]]:
    """Row chunks whose starts are multiples of ``align`` (a 64-row superstep of the MFMA fragment
    layouts packs independently into a contiguous byte range of the image)."""
    step = max(align, (chunk_rows // align) * align)
    for lo in range(0, n, step):
        yield lo, min(n, lo + step)


def shard_byte_range(data: bytes, rank: int, world: int):
    from ..ops.csvscan import shard_byte_range as _sbr

    return _sbr(data, rank, world)
