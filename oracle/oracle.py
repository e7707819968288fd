"""ctypes binding of the C oracle (TEST INFRASTRUCTURE -- the parity checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  It runs the CPU restatement of the reference WGSL (see pt_oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

PASS_GBUFFER, PASS_INIT, PASS_FINAL, PASS_MCPT, PASS_RESTIR = 0, 1, 2, 3, 4
PASS_TEMPORAL, PASS_SPATIAL = 5, 6
# the reuse pipeline's PT_1 (x_{k+1} of a hybrid-shiftable sample in pad words 24..27) and PT_4
# (a reused reservoir's stored contribution, pt_oracle.c final_rows)
PASS_INIT_REUSE, PASS_FINAL_REUSE = 11, 12
# ReSTIR GI passes (build-defined; pt_oracle_gi.c)
GI_PASS_INIT, GI_PASS_TEMPORAL, GI_PASS_SPATIAL, GI_PASS_FINAL = 7, 8, 9, 10
GI_WORDS = 16
# build-defined reuse defaults (same as include/ptx.h)
REUSE_RADIUS, REUSE_NEIGHBORS, TEMPORAL_CAP = 30, 3, 20


class Counters(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_uint64), ("instance_xforms", ctypes.c_uint64),
                ("aabb_tests", ctypes.c_uint64), ("tri_tests", ctypes.c_uint64), ("hits", ctypes.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class ReuseParams(ctypes.Structure):
    _fields_ = [("radius", ctypes.c_uint32), ("neighbors", ctypes.c_uint32), ("temporal_cap", ctypes.c_uint32),
                ("hist_valid", ctypes.c_uint32)]


class Inputs(ctypes.Structure):
    _fields_ = [("uniform", ctypes.c_void_p), ("scene", ctypes.c_void_p),
                ("geometry", ctypes.c_void_p), ("accel", ctypes.c_void_p)]


# build variants: "" = the parity oracle; "libm" / "wgsl" = the transcendental-sensitivity
# builds (PTO_TRANSC=1 / 2 in pt_oracle.c), "asan" = the sanitizer build
VARIANTS = {"": "liboracle.so", "libm": "liboracle_libm.so", "wgsl": "liboracle_wgsl.so",
            "wgsl_pow": "liboracle_wgsl_pow.so", "wgsl_sincos": "liboracle_wgsl_sincos.so",
            "asan": "liboracle_asan.so"}


def build(force: bool = False, variant: str = "") -> str:
    path = os.path.join(HERE, VARIANTS[variant])
    srcs = [os.path.join(HERE, f) for f in ("pt_oracle.c", "pt_oracle_gi.c", "pt_oracle.h")]
    if force or not os.path.exists(path) or os.path.getmtime(path) < max(map(os.path.getmtime, srcs)):
        subprocess.run(["make", "-C", HERE, VARIANTS[variant]], check=True, capture_output=True)
    return path


_libs: dict = {}


def lib(variant: str = ""):
    _lib = _libs.get(variant)
    if _lib is None:
        _lib = _libs[variant] = ctypes.CDLL(build(variant=variant))
        P = ctypes.c_void_p
        _lib.pto_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(Inputs), ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, P, P, P, ctypes.POINTER(Counters)]
        _lib.pto_run.restype = ctypes.c_int
        _lib.pto_run_reuse.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(Inputs), ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P,
                                       ctypes.POINTER(ReuseParams), ctypes.POINTER(Counters)]
        _lib.pto_run_reuse.restype = ctypes.c_int
        _lib.pto_run_temporal_motion.argtypes = [ctypes.c_int, ctypes.POINTER(Inputs), ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_int, P, P, P, P, P,
                                                 ctypes.POINTER(ReuseParams), ctypes.POINTER(Counters)]
        _lib.pto_run_temporal_motion.restype = ctypes.c_int
        _lib.pto_mat4_inverse.argtypes = [P, P]
        _lib.pto_run_gi.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(Inputs), ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, P, P, P, P, P, ctypes.POINTER(ReuseParams),
                                    ctypes.POINTER(Counters)]
        _lib.pto_run_gi.restype = ctypes.c_int
        _lib.pto_run_gi_temporal_motion.argtypes = _lib.pto_run_temporal_motion.argtypes
        _lib.pto_run_gi_temporal_motion.restype = ctypes.c_int
        _lib.pto_gi_shift.argtypes = [ctypes.POINTER(Inputs), P, ctypes.c_uint32, ctypes.c_uint32, P, P]
        _lib.pto_gi_sample_dir.argtypes = [P, P, P, ctypes.POINTER(ctypes.c_uint32), P]
        _lib.pto_gi_sample_dir.restype = ctypes.c_float
        _lib.pto_pcg.argtypes = [ctypes.c_uint32]
        _lib.pto_pcg.restype = ctypes.c_uint32
        _lib.pto_random.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        _lib.pto_random.restype = ctypes.c_float
        for fn in ("pto_sin", "pto_cos", "pto_pow5"):
            getattr(_lib, fn).argtypes = [ctypes.c_float]
            getattr(_lib, fn).restype = ctypes.c_float
        _lib.pto_bsdf.argtypes = [P, P, P, P, P]
        _lib.pto_pdf_bsdf.argtypes = [P, P, P, P]
        _lib.pto_pdf_bsdf.restype = ctypes.c_float
        _lib.pto_sample_bsdf.argtypes = [P, P, P, ctypes.POINTER(ctypes.c_uint32), P,
                                         ctypes.POINTER(ctypes.c_uint32)]
        _lib.pto_trace.argtypes = [ctypes.POINTER(Inputs), P, P, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.POINTER(Counters)]
        _lib.pto_ray_triangle.argtypes = [P, P, P, P, P, ctypes.c_float]
        _lib.pto_ray_triangle.restype = ctypes.c_float
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class Frame:
    """Full-frame oracle buffers for one W x H uniform block."""

    def __init__(self, uniform: np.ndarray, scene: np.ndarray, geometry: np.ndarray, accel: np.ndarray,
                 variant: str = ""):
        self.variant = variant  # oracle build (VARIANTS); "" = the parity oracle
        self.uniform = np.ascontiguousarray(uniform, dtype=np.uint32)
        self.scene = np.ascontiguousarray(scene, dtype=np.uint32)
        self.geometry = np.ascontiguousarray(geometry, dtype=np.uint32)
        self.accel = np.ascontiguousarray(accel, dtype=np.uint32) if len(accel) else np.zeros(1, np.uint32)
        self.W, self.H = int(self.uniform[0]), int(self.uniform[1])
        self.gbuffer = np.zeros((self.H, self.W, 4), dtype=np.uint32)
        self.reservoir = np.zeros((self.H, self.W, 32), dtype=np.uint32)
        self.accum = np.zeros((self.H, self.W, 4), dtype=np.float32)
        self.res_hist = np.zeros((self.H, self.W, 32), dtype=np.uint32)  # spatial output / history
        self.hist_valid = False
        # the frame the history was rendered with (temporal reuse under camera motion: its
        # uniform words -- camera -- and G-buffer; pto_run_temporal_motion)
        self.prev_uniform = self.uniform.copy()
        self.prev_gbuffer = np.zeros_like(self.gbuffer)
        self.reuse = (REUSE_RADIUS, REUSE_NEIGHBORS, TEMPORAL_CAP)
        # ReSTIR GI buffers: candidate / temporal reservoirs, spatial output (= history), direct light
        self.gi_res = np.zeros((self.H, self.W, GI_WORDS), dtype=np.uint32)
        self.gi_hist = np.zeros((self.H, self.W, GI_WORDS), dtype=np.uint32)
        self.direct = np.zeros((self.H, self.W, 4), dtype=np.float32)
        self.counters = {}

    def set_frame_index(self, f: int):
        self.uniform[23] = f

    def set_camera(self, uniform: np.ndarray):
        """A new camera (the uniform's words 4..22: VP^-1 and position); the history stays (it
        is reprojected: motion_moved)."""
        self.uniform[4:23] = np.asarray(uniform, dtype=np.uint32)[4:23]

    def camera_moved(self) -> bool:
        return bool(np.any(self.uniform[4:23] != self.prev_uniform[4:23]))

    def run_temporal_motion(self, threads: int = 0, rect=None) -> dict:
        """Temporal reuse with the history at each pixel's reprojection in the previous frame
        (prev_uniform, prev_gbuffer; pt_oracle.c temporal_motion_pixel)."""
        threads = threads or os.cpu_count() or 1
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, self.W, self.H)
        r, m, cap = self.reuse
        prm = ReuseParams(r, m, cap, 1 if self.hist_valid else 0)
        cnt = Counters()
        rc = lib(self.variant).pto_run_temporal_motion(threads, ctypes.byref(self._inputs()), x0, y0, x1, y1,
                                                      _ptr(self.gbuffer), _ptr(self.reservoir), _ptr(self.res_hist),
                                                      _ptr(self.prev_uniform), _ptr(self.prev_gbuffer),
                                                      ctypes.byref(prm), ctypes.byref(cnt))
        if rc != 0:
            raise RuntimeError(f"oracle motion temporal pass failed ({rc})")
        self.counters["temporal_motion"] = cnt.as_dict()
        return self.counters["temporal_motion"]

    def trace(self, rays: np.ndarray, eps_mode: int = 1, return_counters: bool = False):
        """Closest hits for (n, 8) f32 rays, same format as ptx_trace (+ the traversal work)."""
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        hits = np.zeros_like(rays)
        inp = Inputs(self.uniform.ctypes.data, self.scene.ctypes.data, self.geometry.ctypes.data,
                     self.accel.ctypes.data)
        cnt = Counters()
        lib(self.variant).pto_trace(ctypes.byref(inp), _ptr(rays), _ptr(hits), len(rays), eps_mode, ctypes.byref(cnt))
        self.counters["trace"] = cnt.as_dict()
        return (hits, self.counters["trace"]) if return_counters else hits

    def run(self, pass_id: int, threads: int = 0, rect=None, reservoir: np.ndarray | None = None) -> dict:
        """One pass over `rect` (x0, y0, x1, y1).  PASS_TEMPORAL updates `reservoir` from
        `res_hist`; PASS_SPATIAL reads `reservoir` and writes `res_hist`; PASS_FINAL reads
        `reservoir` (pass `reservoir=self.res_hist` for the reuse pipeline)."""
        threads = threads or os.cpu_count() or 1
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, self.W, self.H)
        inp = Inputs(self.uniform.ctypes.data, self.scene.ctypes.data, self.geometry.ctypes.data,
                     self.accel.ctypes.data)
        cnt = Counters()
        if pass_id in (PASS_TEMPORAL, PASS_SPATIAL):
            r, m, cap = self.reuse
            prm = ReuseParams(r, m, cap, 1 if self.hist_valid else 0)
            rc = lib(self.variant).pto_run_reuse(pass_id, threads, ctypes.byref(inp), x0, y0, x1, y1, _ptr(self.gbuffer),
                                     _ptr(self.reservoir), _ptr(self.res_hist), ctypes.byref(prm),
                                     ctypes.byref(cnt))
            if rc != 0:
                raise RuntimeError(f"oracle pass {pass_id} failed ({rc})")
            self.counters[pass_id] = cnt.as_dict()
            return self.counters[pass_id]
        res = self.reservoir if reservoir is None else np.ascontiguousarray(reservoir)
        assert res.dtype == np.uint32 and res.shape == self.reservoir.shape
        rc = lib(self.variant).pto_run(pass_id, threads, ctypes.byref(inp), x0, y0, x1, y1, _ptr(self.gbuffer),
                           _ptr(res), _ptr(self.accum), ctypes.byref(cnt))
        if rc != 0:
            raise RuntimeError(f"oracle pass {pass_id} failed ({rc})")
        self.counters[pass_id] = cnt.as_dict()
        return self.counters[pass_id]

    def run_reuse_frame(self, threads: int = 0, rect=None) -> None:
        """One frame of the reuse pipeline: G-buffer -> PT_1 -> temporal -> spatial -> PT_4.
        A camera moved since the history's frame (set_camera) reprojects the history
        (run_temporal_motion) instead of the same-pixel temporal pass; clearing `hist_valid`
        drops it (ptx_upload_scene / ptx_reset_accumulation do)."""
        moved = self.hist_valid and self.camera_moved()
        for p in (PASS_GBUFFER, PASS_INIT_REUSE):
            self.run(p, threads, rect)
        if moved:
            self.run_temporal_motion(threads, rect)
        else:
            self.run(PASS_TEMPORAL, threads, rect)
        self.run(PASS_SPATIAL, threads, rect)
        self.run(PASS_FINAL_REUSE, threads, rect, reservoir=self.res_hist)
        self.hist_valid = True
        self.prev_uniform = self.uniform.copy()
        self.prev_gbuffer[...] = self.gbuffer


    def run_reuse_frame_census(self, threads: int = 0) -> np.ndarray:
        """run_reuse_frame, pass by pass over one 8-row tile row at a time: returns the
        (tile rows, 5) work {rays, instance transforms, AABB tests, triangle tests, hits} of
        every query traced for each tile row's pixels (ptx_row_census's counters).  Every
        pass reads only the previous passes' complete outputs (the spatial pass the temporal
        output of all rows), so the frame is the same as run_reuse_frame's."""
        T = (self.H + 7) // 8
        out = np.zeros((T, 5), dtype=np.uint64)
        keys = ("rays", "instance_xforms", "aabb_tests", "tri_tests", "hits")
        for p in (PASS_GBUFFER, PASS_INIT_REUSE, PASS_TEMPORAL, PASS_SPATIAL, PASS_FINAL_REUSE):
            for t in range(T):
                rect = (0, 8 * t, self.W, min(self.H, 8 * t + 8))
                c = self.run(p, threads, rect, reservoir=self.res_hist if p == PASS_FINAL_REUSE else None)
                out[t] += np.array([c[k] for k in keys], dtype=np.uint64)
        self.hist_valid = True
        return out

    def _inputs(self):
        return Inputs(self.uniform.ctypes.data, self.scene.ctypes.data, self.geometry.ctypes.data,
                      self.accel.ctypes.data)

    def run_gi(self, pass_id: int, threads: int = 0, rect=None) -> dict:
        """One ReSTIR GI pass (GI_PASS_*) over `rect`: init writes gi_res + direct, temporal
        updates gi_res from gi_hist, spatial writes gi_hist, final accumulates into accum."""
        threads = threads or os.cpu_count() or 1
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, self.W, self.H)
        r, m, cap = self.reuse
        prm = ReuseParams(r, m, cap, 1 if self.hist_valid else 0)
        cnt = Counters()
        inp = self._inputs()
        rc = lib(self.variant).pto_run_gi(pass_id, threads, ctypes.byref(inp), x0, y0, x1, y1, _ptr(self.gbuffer),
                              _ptr(self.gi_res), _ptr(self.gi_hist), _ptr(self.direct), _ptr(self.accum),
                              ctypes.byref(prm), ctypes.byref(cnt))
        if rc != 0:
            raise RuntimeError(f"oracle GI pass {pass_id} failed ({rc})")
        self.counters[("gi", pass_id)] = cnt.as_dict()
        return self.counters[("gi", pass_id)]

    def run_gi_temporal_motion(self, threads: int = 0, rect=None) -> dict:
        """GI temporal reuse with the history at each pixel's reprojection in the previous frame
        (prev_uniform, prev_gbuffer; pt_oracle_gi.c gi_temporal_motion_pixel)."""
        threads = threads or os.cpu_count() or 1
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, self.W, self.H)
        r, m, cap = self.reuse
        prm = ReuseParams(r, m, cap, 1 if self.hist_valid else 0)
        cnt = Counters()
        rc = lib(self.variant).pto_run_gi_temporal_motion(threads, ctypes.byref(self._inputs()), x0, y0, x1, y1,
                                                         _ptr(self.gbuffer), _ptr(self.gi_res), _ptr(self.gi_hist),
                                                         _ptr(self.prev_uniform), _ptr(self.prev_gbuffer),
                                                         ctypes.byref(prm), ctypes.byref(cnt))
        if rc != 0:
            raise RuntimeError(f"oracle GI motion temporal pass failed ({rc})")
        self.counters["gi_temporal_motion"] = cnt.as_dict()
        return self.counters["gi_temporal_motion"]

    def run_gi_frame(self, threads: int = 0, rect=None) -> None:
        """One ReSTIR GI frame: G-buffer -> GI init -> temporal -> spatial -> shade.  As in
        run_reuse_frame, a camera moved since the history's frame reprojects the history
        (run_gi_temporal_motion)."""
        moved = self.hist_valid and self.camera_moved()
        self.run(PASS_GBUFFER, threads, rect)
        self.run_gi(GI_PASS_INIT, threads, rect)
        if moved:
            self.run_gi_temporal_motion(threads, rect)
        else:
            self.run_gi(GI_PASS_TEMPORAL, threads, rect)
        for p in (GI_PASS_SPATIAL, GI_PASS_FINAL):
            self.run_gi(p, threads, rect)
        self.hist_valid = True
        self.prev_uniform = self.uniform.copy()
        self.prev_gbuffer[...] = self.gbuffer

    def gi_shift(self, x: int, y: int, s: np.ndarray):
        """The GI reconnection shift of reservoir `s` (16 words) into pixel (x, y):
        (valid, f rgb, q)."""
        s = np.ascontiguousarray(s, dtype=np.uint32)
        out = np.zeros(5, dtype=np.float32)
        inp = self._inputs()
        lib(self.variant).pto_gi_shift(ctypes.byref(inp), _ptr(self.gbuffer), x, y, _ptr(s), _ptr(out))
        return bool(out[0]), out[1:4].copy(), float(out[4])


def present(img: np.ndarray, canvas_w: int, canvas_h: int, bgra: bool = False) -> np.ndarray:
    """Renderer_TEST.Render's render pass (GC/Renderer_TEST.ts:233-255): the fullscreen quad of
    VertexShader.wgsl (PixelUV = (NDC + 1) / 2) and FragmentShader.wgsl:7-10 (texel
    (floor(PixelUV.x * 600), floor(PixelUV.y * 450)) of the Scene texture, rgb, alpha 1) onto a
    unorm8 canvas; canvas row 0 is the top (NDC y = +1).  `img`: the (H, W, 4) f32 texture, row 0 =
    image row 0.  Exact integer texel arithmetic; out-of-bounds texels read 0; unorm8 = clamp to
    [0, 1], x * 255 rounded half to even, NaN -> 0 (test restatement of ptx_present)."""
    H, W = img.shape[:2]
    px = np.arange(canvas_w, dtype=np.int64)
    py = np.arange(canvas_h, dtype=np.int64)
    tx = ((2 * px + 1) * 600) // (2 * canvas_w)
    ty = ((2 * canvas_h - 2 * py - 1) * 450) // (2 * canvas_h)
    out = np.zeros((canvas_h, canvas_w, 4), np.uint8)
    ok = (ty[:, None] < H) & (tx[None, :] < W)
    rgb = np.zeros((canvas_h, canvas_w, 3), np.float32)
    yy, xx = np.broadcast_arrays(ty[:, None], tx[None, :])
    rgb[ok] = img[yy[ok], xx[ok], :3]
    c = np.nan_to_num(rgb, nan=0.0)
    c = np.clip(c, np.float32(0.0), np.float32(1.0))
    q = np.rint(c * np.float32(255.0)).astype(np.uint8)
    out[..., :3] = q[..., ::-1] if bgra else q
    out[..., 3] = 255
    return out


def pcg(seed: int) -> int:
    return int(lib().pto_pcg(seed & 0xFFFFFFFF))


def fixed_sin(x: float) -> float:
    """The fixed f32 sin both sides use for BSDF sampling angles (x >= 0)."""
    return float(lib().pto_sin(x))


def fixed_cos(x: float) -> float:
    return float(lib().pto_cos(x))


def fixed_pow5(x: float) -> float:
    return float(lib().pto_pow5(x))


def bsdf(n, mat, v, l) -> np.ndarray:
    args = [np.asarray(a, dtype=np.float32) for a in (n, mat, v, l)]
    out = np.zeros(3, dtype=np.float32)
    lib().pto_bsdf(*[_ptr(a) for a in args], _ptr(out))
    return out


def pdf_bsdf(n, mat, v, l) -> float:
    args = [np.asarray(a, dtype=np.float32) for a in (n, mat, v, l)]
    return float(lib().pto_pdf_bsdf(*[_ptr(a) for a in args]))


def sample_bsdf(n, mat, v, seed: int):
    args = [np.asarray(a, dtype=np.float32) for a in (n, mat, v)]
    s = ctypes.c_uint32(seed)
    lobe = ctypes.c_uint32(0)
    out = np.zeros(3, dtype=np.float32)
    lib().pto_sample_bsdf(*[_ptr(a) for a in args], ctypes.byref(s), _ptr(out), ctypes.byref(lobe))
    return out, int(lobe.value), int(s.value)


def gi_sample_dir(n, mat, v, seed: int):
    """The GI candidate sampler: (direction, pdf, next seed)."""
    args = [np.asarray(a, dtype=np.float32) for a in (n, mat, v)]
    s = ctypes.c_uint32(seed)
    out = np.zeros(3, dtype=np.float32)
    pdf = float(lib().pto_gi_sample_dir(*[_ptr(a) for a in args], ctypes.byref(s), _ptr(out)))
    return out, pdf, int(s.value)


def ray_triangle(o, d, p0, p1, p2, det_eps: float) -> float:
    args = [np.asarray(a, dtype=np.float32) for a in (o, d, p0, p1, p2)]
    return float(lib().pto_ray_triangle(*[_ptr(a) for a in args], det_eps))
