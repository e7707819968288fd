"""Image-space decomposition across ranks.

The reference's passes are independent per pixel (every kernel reads only its own
pixel's G-buffer texel / reservoir), and RNG seeds and camera rays use the *global*
pixel coordinates (SH/PT_1_InitPass.wgsl:823-826, SH/PT_01_GBufferPass.wgsl:496-507),
so any row-band split renders the same image bit for bit.  No collective is needed on
the data path; gathering the image is only for display.
"""
from __future__ import annotations


def band(height: int, world: int, rank: int) -> tuple[int, int]:
    """Strong scaling: rows [begin, end) of a fixed image for `rank` of `world` (balanced)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(height, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def weak_band(rows_per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: every rank owns `rows_per_rank` rows of a (rows_per_rank * world)-row image."""
    return rank * rows_per_rank, (rank + 1) * rows_per_rank
