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
