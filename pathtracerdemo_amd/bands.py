"""Image-space decomposition across ranks.

The reference's passes are independent per pixel (every kernel reads only its own
pixel's G-buffer texel / reservoir), and RNG seeds and camera rays use the *global*
pixel coordinates (SH/PT_1_InitPass.wgsl:823-826, SH/PT_01_GBufferPass.wgsl:496-507),
so any row-band split renders the same image bit for bit.  No collective is needed on
the data path of the reference's passes; gathering the image is only for display.

The reuse pipeline has the one real exchange step: the spatial pass
reads neighbours up to `reuse_radius` rows away, so between the temporal and spatial
passes every band swaps its first / last `radius` rows of G-buffer + reservoirs with the
bands above / below: point-to-point over RCCL (xGMI) with the
nccl backend, gloo on CPU.  `ReuseBand` drives one frame of a band through that.
"""
from __future__ import annotations

import numpy as np


def band(height: int, world: int, rank: int) -> tuple[int, int]:
    """Strong scaling: rows [begin, end) of a fixed image for `rank` of `world` (balanced)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(height, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


# SURVEY.md §8(d)'s algorithmic bytes per counted unit of traversal work: AABB test, triangle
# test, instance transform, hit reconstruction, and the 64-byte ray + hit record per query
CENSUS_BYTES = np.array([64, 48, 32, 36, 48], dtype=np.float64)  # rays, inst, aabb, tri, hits
# fixed per-pixel pass IO of the reuse pipeline (bench.py PASS_IO: G-buffer, PT_1, temporal,
# spatial, PT_4)
REUSE_PIXEL_BYTES = 16 + (16 + 128) + (16 + 3 * 128) + (4 * (16 + 128) + 128) + (16 + 128 + 16 + 16)


def row_costs(tile_census: np.ndarray, width: int, height: int, pixel_bytes: float = REUSE_PIXEL_BYTES) -> np.ndarray:
    """Predicted cost (algorithmic bytes) of every pixel row of a `height`-row frame from a
    tile-row census ((T, 5) counters per 8-row tile row, ptx_row_census / the oracle's
    run_reuse_frame_census) taken on a frame of T*8 >= census rows: each tile row's work is
    spread evenly over its rows, and a census of another height is resampled (same camera,
    so census row r covers frame rows r * height / census_rows ...)."""
    tc = np.asarray(tile_census, dtype=np.float64).reshape(-1, 5) @ CENSUS_BYTES
    per_row = np.repeat(tc / 8.0, 8)  # census pixel rows (the last tile row may be partial)
    n = len(per_row)
    # cumulative cost at census-row boundaries, resampled linearly onto the frame's rows
    cum = np.concatenate([[0.0], np.cumsum(per_row)])
    edges = np.linspace(0.0, n, height + 1)
    cum_f = np.interp(edges, np.arange(n + 1), cum)
    return np.diff(cum_f) + pixel_bytes * width


def balanced_bands(costs, world: int, min_rows: int = 1) -> list[tuple[int, int]]:
    """Row bands [begin, end) covering len(costs) rows that minimise the largest band cost,
    every band holding >= min_rows rows (a reuse band must hold the halo radius).  Exact
    dynamic program over the prefix sums (world x H x H, vectorised over the split row)."""
    c = np.asarray(costs, dtype=np.float64)
    H = len(c)
    if world < 1 or min_rows * world > H:
        raise ValueError(f"cannot split {H} rows into {world} bands of >= {min_rows} rows")
    P = np.concatenate([[0.0], np.cumsum(c)])
    INF = np.inf
    best = np.full(H + 1, INF)  # best[i]: the smallest max-cost covering rows [0, i) with k bands
    best[min_rows:] = P[min_rows:]
    choice = [np.zeros(H + 1, dtype=np.int64)]
    for k in range(2, world + 1):
        nb = np.full(H + 1, INF)
        ch = np.zeros(H + 1, dtype=np.int64)
        for i in range(k * min_rows, H + 1):
            j = np.arange((k - 1) * min_rows, i - min_rows + 1)
            v = np.maximum(best[j], P[i] - P[j])
            a = int(np.argmin(v))
            nb[i], ch[i] = v[a], j[a]
        best = nb
        choice.append(ch)
    bounds = [H]
    i = H
    for k in range(world, 1, -1):
        i = int(choice[k - 1][i])
        bounds.append(i)
    bounds.append(0)
    bounds = bounds[::-1]
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def band_balance(costs, bands) -> float:
    """max / mean predicted band cost (1.0 = perfect)."""
    c = np.asarray(costs, dtype=np.float64)
    v = np.array([c[b:e].sum() for b, e in bands])
    return float(v.max() / v.mean())


def recalibrated_costs(costs, bands, band_ms) -> np.ndarray:
    """Row costs rescaled by measured band time: every row of band b is multiplied by
    band_ms[b] / (its predicted band cost), so each band's rescaled sum IS its measured time
    and the rows keep their census shape inside it.  The census counts algorithmic bytes, and
    rows of the same byte count can differ 2-3x in time (divergent walks, launch tails of a
    small band): on C4 over 8 bands the census's 1.002 predicted max/mean measured 1.36."""
    c = np.asarray(costs, dtype=np.float64).copy()
    for (b0, b1), t in zip(bands, band_ms):
        pred = float(c[b0:b1].sum())
        if pred > 0.0 and t > 0.0:
            c[b0:b1] *= t / pred
    return c


def weak_band(rows_per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: every rank owns `rows_per_rank` rows of a (rows_per_rank * world)-row image."""
    return rank * rows_per_rank, (rank + 1) * rows_per_rank


def halo_exchange(send_top, send_bottom, recv_top, recv_bottom, rank: int, world: int) -> None:
    """Swap halo messages with the neighbouring bands (rank - 1 above, rank + 1 below).

    send_top goes up (it becomes rank-1's bottom halo), send_bottom goes down; recv_top /
    recv_bottom receive the neighbours' messages.  Tensors of a missing neighbour are unused.
    One batched isend/irecv group: with the nccl backend it runs on RCCL's stream after the
    producing kernels of torch's current stream, and the current stream waits for it."""
    import torch.distributed as dist
    ops = []
    if rank > 0 and send_top.numel():
        ops += [dist.P2POp(dist.isend, send_top, rank - 1), dist.P2POp(dist.irecv, recv_top, rank - 1)]
    if rank < world - 1 and send_bottom.numel():
        ops += [dist.P2POp(dist.isend, send_bottom, rank + 1), dist.P2POp(dist.irecv, recv_bottom, rank + 1)]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


class ReuseBand:
    """One rank's band of the reuse pipeline: the frame as two pass groups around the halo
    exchange.  `target` is a Renderer(pipeline="reuse", row_begin, row_end) -- or any object
    with its run_passes / halo_rows / halo_pack / halo_unpack methods (the CPU tests drive
    the oracle through the same class).  Buffers are uint8 tensors on `device`; their
    data_ptr() is what halo_pack / halo_unpack see."""

    FRONT = (0, 1, 8)  # PTX_PASS_GBUFFER, PTX_PASS_INIT, PTX_PASS_TEMPORAL
    BACK = (9, 2)      # PTX_PASS_SPATIAL, PTX_PASS_FINAL

    def __init__(self, target, rank: int, world: int, device="cpu"):
        import torch
        self.t, self.rank, self.world = target, rank, world
        self.host_buffers = not str(device).startswith("cuda")
        if not self.host_buffers:  # pack -> RCCL -> unpack ordered on torch's stream
            target.set_stream(torch.cuda.current_stream(device).cuda_stream)
        top, bottom, row_bytes = target.halo_rows()
        mk = lambda rows: torch.empty(rows * row_bytes, dtype=torch.uint8, device=device)
        self.send_top, self.recv_top = mk(top), mk(top)
        self.send_bottom, self.recv_bottom = mk(bottom), mk(bottom)

    @staticmethod
    def _ptr(t):
        return t.data_ptr() if t.numel() else None

    def render_frame(self) -> None:
        t = self.t
        t.run_passes(self.FRONT)
        t.halo_pack(self._ptr(self.send_top), self._ptr(self.send_bottom))
        if self.host_buffers and hasattr(t, "synchronize"):
            t.synchronize()  # host messages (gloo): the copies must land before sending
        halo_exchange(self.send_top, self.send_bottom, self.recv_top, self.recv_bottom, self.rank, self.world)
        t.halo_unpack(self._ptr(self.recv_top), self._ptr(self.recv_bottom))
        t.run_passes(self.BACK)
