"""Host-side mirror of the reference renderer class over the HIP C ABI.

Same surface and semantics as ``Renderer`` of apps/frontend/src/graphics-core/
Renderer_TEST.ts (constructor :83-126, GetCamera :129-132, ResetFrameCount :134-137,
Initialize :141-163, Update :165-206, Render :208-261), with the WebGPU device replaced
by libptx.so on one MI355X.  ``pipeline="mcpt"`` mirrors the legacy Renderer.ts
(TEST_MCPT.wgsl brute force, GC/Renderer.ts:536-647); ``pipeline="reuse"`` adds the
build-defined temporal + spatial reuse passes between PT_1 and PT_4;
``pipeline="gi"`` is BASELINE configs[4], ReSTIR GI.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from .scene.camera import Camera
from .scene.world import CompiledScene, World, serialize_world


class Renderer:
    def __init__(self, width: int, height: int, device: int = -1, pipeline: str = "restir",
                 row_begin: int = 0, row_end: int = 0, count_work: bool = False, variant: str = "wave",
                 time_launches: bool = False, single_stream: bool = False, reuse_radius: int = 0,
                 reuse_neighbors: int = 0, temporal_cap: int = 0, row_census: bool = False,
                 halo_overlap: bool = False, halo_skip: bool = False):
        self._lib = N.load()
        self.width, self.height = int(width), int(height)
        self.pipeline = pipeline
        cfg = N.PtxConfig(width=self.width, height=self.height, row_begin=row_begin, row_end=row_end,
                          device=device,
                          pipeline=N.PIPELINES[pipeline], reuse_radius=reuse_radius,
                          reuse_neighbors=reuse_neighbors, temporal_cap=temporal_cap,
                          flags=(N.PTX_FLAG_COUNT_WORK if count_work else 0) | N.VARIANT_FLAGS[variant]
                          | (N.PTX_FLAG_TIME_LAUNCHES if time_launches else 0)
                          | (N.PTX_FLAG_SINGLE_STREAM if single_stream else 0)
                          | (N.PTX_FLAG_ROW_CENSUS if row_census else 0)
                          | (N.PTX_FLAG_HALO_OVERLAP if halo_overlap else 0)
                          | (N.PTX_FLAG_HALO_SKIP if halo_skip else 0))
        self._h = ctypes.c_void_p()
        rc = self._lib.ptx_create(ctypes.byref(cfg), ctypes.byref(self._h))
        if rc != N.PTX_OK:
            raise N.PtxError(f"ptx_create failed ({rc})")
        self.row_begin = row_begin
        self.row_end = row_end or self.height
        self.compiled: CompiledScene | None = None
        self.camera: Camera | None = None
        self.frame_count = 0
        self.uniform = None

    # ------------------------------------------------------------------ reference surface
    def GetCamera(self) -> Camera:
        return self.camera

    def ResetFrameCount(self) -> None:
        self.frame_count = 0

    def Initialize(self, world: World | CompiledScene) -> None:
        """Renderer_TEST.Initialize: camera at (0,0,6), yaw/pitch 0, FrameCount 0, upload."""
        self.camera = Camera(self.width, self.height)
        self.camera.set_location(0, 0, 6)
        self.camera.set_yaw(0)
        self.camera.set_pitch(0)
        self.ResetFrameCount()
        self.compiled = world if isinstance(world, CompiledScene) else serialize_world(world)
        cs = self.compiled
        self._call("ptx_upload_scene", self._h, cs.scene.ctypes.data, len(cs.scene), cs.geometry.ctypes.data,
                   len(cs.geometry), cs.accel.ctypes.data if len(cs.accel) else None, len(cs.accel))
        self._call("ptx_reset_accumulation", self._h)

    def Update(self) -> None:
        """Renderer_TEST.Update: FrameCount++ and the 33-word uniform block."""
        self.frame_count += 1
        u = self.compiled.uniform(self.width, self.height, self.camera.view_projection_inverse(),
                                  self.camera.location, self.frame_count)
        self.set_uniform(u)

    def Render(self) -> None:
        """Renderer_TEST.Render: the configured passes, accumulated into the Scene texture."""
        self._call("ptx_render", self._h, None)

    # ------------------------------------------------------------------ extras
    def set_uniform(self, u: np.ndarray) -> None:
        self.uniform = np.ascontiguousarray(u, dtype=np.uint32)
        self._call("ptx_set_frame", self._h, self.uniform.ctypes.data)

    def run_pass(self, pass_id: int) -> None:
        self._call("ptx_run_pass", self._h, pass_id)

    def run_passes(self, passes) -> None:
        """Several passes as one overlapped launch sequence (include/ptx.h ptx_run_passes)."""
        arr = (ctypes.c_int * len(passes))(*passes)
        self._call("ptx_run_passes", self._h, arr, len(passes))

    def halo_rows(self):
        """(rows above, rows below, bytes per halo row) of a reuse band (ptx_halo_rows)."""
        t, b, n = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_size_t()
        self._call("ptx_halo_rows", self._h, ctypes.byref(t), ctypes.byref(b), ctypes.byref(n))
        return int(t.value), int(b.value), int(n.value)

    def halo_pack(self, dev_top: int | None, dev_bottom: int | None) -> None:
        self._call("ptx_halo_pack", self._h, dev_top, dev_bottom)

    def halo_unpack(self, dev_top: int | None, dev_bottom: int | None) -> None:
        self._call("ptx_halo_unpack", self._h, dev_top, dev_bottom)

    # ------------------------------------------------------------------ multi-GPU (include/ptx.h)
    @staticmethod
    def comm_unique_id() -> bytes:
        """ncclGetUniqueId: made on one rank, shipped to the others by the caller."""
        lib = N.load()
        buf = ctypes.create_string_buffer(N.PTX_COMM_ID_BYTES)
        rc = lib.ptx_comm_unique_id(buf, N.PTX_COMM_ID_BYTES)
        if rc != N.PTX_OK:
            raise N.PtxError(f"ptx_comm_unique_id failed ({rc}): is RCCL installed?")
        return buf.raw

    def comm_init(self, unique_id: bytes, rank: int, world: int) -> None:
        """The handle's own RCCL communicator: Render() then exchanges the halo itself."""
        buf = ctypes.create_string_buffer(bytes(unique_id), N.PTX_COMM_ID_BYTES)
        self._call("ptx_comm_init", self._h, buf, N.PTX_COMM_ID_BYTES, rank, world)

    def comm_info(self) -> dict:
        """The handle's communicator: rank, world size (1 without one), halo bytes sent so far."""
        rank, world, sent = ctypes.c_int(0), ctypes.c_int(1), ctypes.c_uint64(0)
        self._call("ptx_comm_info", self._h, ctypes.byref(rank), ctypes.byref(world), ctypes.byref(sent))
        return {"rank": rank.value, "world": world.value, "halo_bytes_sent": sent.value}

    @staticmethod
    def comm_init_all(renderers) -> None:
        """ncclCommInitAll over the band renderers of this process (one per GPU)."""
        arr = (ctypes.c_void_p * len(renderers))(*[r._h.value for r in renderers])
        lib = N.load()
        N.check(lib, renderers[0]._h, lib.ptx_comm_init_all(arr, len(renderers)), "ptx_comm_init_all")

    @staticmethod
    def render_bands(renderers, out: np.ndarray | None = None) -> None:
        """One frame over the band renderers of this process, halo exchanged on the device
        (their communicators, or peer copies); `out` (rows of all bands, W, 4) f32 optional."""
        arr = (ctypes.c_void_p * len(renderers))(*[r._h.value for r in renderers])
        lib = N.load()
        ptr = None
        if out is not None:
            rows = sum(r.band_rows for r in renderers)
            assert out.dtype == np.float32 and out.flags.c_contiguous and out.size == rows * renderers[0].width * 4
            ptr = out.ctypes.data
        rc = lib.ptx_render_bands(arr, len(renderers), ptr)
        if rc != N.PTX_OK:
            msgs = [lib.ptx_last_error(r._h) for r in renderers]
            raise N.PtxError(f"ptx_render_bands failed ({rc}): "
                             + "; ".join(m.decode(errors="replace") for m in msgs if m))

    def row_census(self) -> np.ndarray:
        """(tile rows, 5) u64 {rays, instance transforms, AABB tests, triangle tests, hits}
        per 8-row tile row of the band (handle made with row_census=True)."""
        out = np.zeros(((self.band_rows + 7) // 8, 5), dtype=np.uint64)
        self._call("ptx_row_census", self._h, out.ctypes.data, out.shape[0])
        return out

    @property
    def reservoir_words(self) -> int:
        """32 (the reference's 128-byte Reservoir) or 16 (the GI reservoir)."""
        return 16 if self.pipeline == "gi" else 32

    def read_history(self) -> np.ndarray:
        """The reuse / GI pipeline's spatial output (final pass input, next frame's history)."""
        return self._read(N.PTX_BUF_RESERVOIR_HIST, np.uint32, self.reservoir_words)

    def read_direct(self) -> np.ndarray:
        """The GI init pass's direct light (band_h, W, 4) f32."""
        return self._read(N.PTX_BUF_DIRECT, np.float32, 4)

    def synchronize(self) -> None:
        self._call("ptx_synchronize", self._h)

    def reset_accumulation(self) -> None:
        self._call("ptx_reset_accumulation", self._h)

    @property
    def band_rows(self) -> int:
        return self.row_end - self.row_begin

    def _read(self, which: int, dtype, comps: int) -> np.ndarray:
        out = np.zeros((self.band_rows, self.width, comps), dtype=dtype)
        self._call("ptx_read_buffer", self._h, which, out.ctypes.data, out.nbytes)
        return out

    def read_image(self) -> np.ndarray:
        return self._read(N.PTX_BUF_ACCUM, np.float32, 4)

    def read_gbuffer(self) -> np.ndarray:
        return self._read(N.PTX_BUF_GBUFFER, np.uint32, 4)

    def read_reservoir(self) -> np.ndarray:
        return self._read(N.PTX_BUF_RESERVOIR, np.uint32, self.reservoir_words)

    def write_buffer(self, which: int, arr: np.ndarray) -> None:
        arr = np.ascontiguousarray(arr)
        self._call("ptx_write_buffer", self._h, which, arr.ctypes.data, arr.nbytes)

    def read_counters(self) -> dict:
        c = np.zeros(8, dtype=np.uint64)
        self._call("ptx_read_buffer", self._h, N.PTX_BUF_COUNTERS, c.ctypes.data, c.nbytes)
        # cull_misses: queries of the counting build whose instance cull would have skipped an
        # instance with a root its pre-filter passes (the cull's conservativeness check: always 0)
        return {"rays": int(c[0]), "instance_xforms": int(c[1]), "aabb_tests": int(c[2]), "tri_tests": int(c[3]),
                "hits": int(c[4]), "cull_misses": int(c[5]),
                # motion_clips (every build): pixels of a moved camera's frames whose reprojection
                # fell past a band's motion halo (no history there; 0 keeps bands bit-identical)
                "motion_clips": int(c[N.PTX_COUNTER_MOTION_CLIP])}

    def stats(self) -> dict:
        s = N.PtxStats()
        self._call("ptx_get_stats", self._h, ctypes.byref(s))
        return {"frames": s.frames, "kernel_ms_total": list(s.kernel_ms_total),
                "kernel_launches": list(s.kernel_launches), "triangles": s.triangles, "bvh_nodes": s.bvh_nodes,
                "instances": s.instances, "max_bvh_depth": s.max_bvh_depth, "device_bytes": s.device_bytes}

    def Present(self, canvas_w: int | None = None, canvas_h: int | None = None, bgra: bool = False) -> np.ndarray:
        """The reference's render pass (Renderer_TEST.Render's fullscreen quad + FragmentShader.wgsl)
        onto a canvas_w x canvas_h canvas (default: the image size): (canvas_h, canvas_w, 4) uint8,
        RGBA (a 2D canvas's ImageData) or BGRA (a bgra8unorm WebGPU canvas); include/ptx.h ptx_present."""
        cw, ch = int(canvas_w or self.width), int(canvas_h or self.height)
        out = np.zeros((ch, cw, 4), np.uint8)
        self._call("ptx_present", self._h, cw, ch, 1 if bgra else 0, out.ctypes.data)
        return out

    def present_async(self, canvas_w: int | None = None, canvas_h: int | None = None, bgra: bool = False) -> None:
        """Enqueue Present for the frame last rendered without waiting (ptx_present_async);
        present_poll() returns the bytes once they have landed."""
        cw, ch = int(canvas_w or self.width), int(canvas_h or self.height)
        self._call("ptx_present_async", self._h, cw, ch, 1 if bgra else 0)
        self._present_shape = (ch, cw, 4)

    def present_poll(self) -> np.ndarray | None:
        """The bytes of the present in flight, or None while it is still running (never waits)."""
        out = np.zeros(self._present_shape, np.uint8)
        rc = self._lib.ptx_present_poll(self._h, out.ctypes.data, out.nbytes)
        if rc == N.PTX_E_PENDING:
            return None
        N.check(self._lib, self._h, rc, "ptx_present_poll")
        return out

    def trace(self, rays: np.ndarray, eps_mode: int = 1) -> np.ndarray:
        """Closest hits for an (n, 8) f32 ray array {o.xyz, d.xyz, -, -}; returns (n, 8) f32
        {t, flags|inst|mat bits, prim bits, bary.x, bary.y, pos.xyz} (include/ptx.h)."""
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        hits = np.zeros_like(rays)
        self._call("ptx_trace", self._h, rays.ctypes.data, hits.ctypes.data, len(rays), eps_mode)
        return hits

    def reset_stats(self) -> None:
        self._call("ptx_reset_stats", self._h)

    def set_stream(self, stream_ptr: int | None) -> None:
        self._call("ptx_set_stream", self._h, stream_ptr)

    def close(self) -> None:
        if self._h:
            self._lib.ptx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _call(self, name: str, *args):
        N.check(self._lib, self._h, getattr(self._lib, name)(*args), name)
