"""ctypes binding of libptx.so (the C ABI of include/ptx.h).

The product path: if the HIP library is missing or fails to load, importing the
renderer raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# PTX_LIB_PATH overrides the in-tree library (same-box A/B of two builds); it must still exist
LIB_PATH = os.environ.get("PTX_LIB_PATH") or os.path.join(PKG_DIR, "libptx.so")

PTX_OK = 0
PTX_E_PENDING = -5  # ptx_present_poll: still in flight
PTX_ABI_VERSION = 5
PTX_PIPELINE_RESTIR, PTX_PIPELINE_MCPT, PTX_PIPELINE_RESTIR_REUSE, PTX_PIPELINE_RESTIR_GI = 0, 1, 2, 3
PIPELINES = {"restir": PTX_PIPELINE_RESTIR, "mcpt": PTX_PIPELINE_MCPT, "reuse": PTX_PIPELINE_RESTIR_REUSE,
             "gi": PTX_PIPELINE_RESTIR_GI}
PTX_PASS_GBUFFER, PTX_PASS_INIT, PTX_PASS_FINAL, PTX_PASS_MCPT, PTX_PASS_TRACE = 0, 1, 2, 3, 4
PTX_PASS_TEMPORAL, PTX_PASS_SPATIAL = 8, 9
PTX_STAT_WAVE_TRACE, PTX_STAT_WAVE_LOGIC, PTX_STAT_FRAME = 5, 6, 7  # stats-only slots (include/ptx.h)
PTX_STAT_PASS_GROUP = 10
PTX_STAT_FINAL_FUSED = 11
PTX_BUF_GBUFFER, PTX_BUF_RESERVOIR, PTX_BUF_ACCUM, PTX_BUF_COUNTERS, PTX_BUF_RESERVOIR_HIST = 0, 1, 2, 3, 4
PTX_BUF_DIRECT = 5
PTX_COUNTER_MOTION_CLIP = 6  # word of PTX_BUF_COUNTERS: pixels a band could not reproject (ptx.h)
PTX_FLAG_COUNT_WORK = 1
PTX_FLAG_SIMPLE_KERNELS = 2
PTX_FLAGS_RETIRED = 12  # the removed persistent-lane / tiled A/B variants: ptx_create rejects them
PTX_FLAG_TIME_LAUNCHES = 16
PTX_FLAG_SINGLE_STREAM = 32
PTX_FLAG_ROW_CENSUS = 64
PTX_FLAG_HALO_OVERLAP = 128
PTX_FLAG_HALO_SKIP = 256  # band frame without the exchange: timing only (edge rows are not the split frame's)
PTX_COMM_ID_BYTES = 128
VARIANT_FLAGS = {"wave": 0, "simple": PTX_FLAG_SIMPLE_KERNELS}

# every symbol include/ptx.h declares (checked by tests/test_abi.py)
EXPORTED = ["ptx_abi_version", "ptx_create", "ptx_upload_scene", "ptx_set_frame", "ptx_render", "ptx_run_pass",
            "ptx_reset_accumulation", "ptx_synchronize", "ptx_get_stats", "ptx_reset_stats", "ptx_read_buffer",
            "ptx_write_buffer", "ptx_device_pointer", "ptx_set_stream", "ptx_destroy", "ptx_last_error",
            "ptx_trace", "ptx_trace_device", "ptx_run_passes", "ptx_halo_rows", "ptx_halo_pack",
            "ptx_halo_unpack", "ptx_comm_unique_id", "ptx_comm_init", "ptx_comm_init_all", "ptx_render_bands",
            "ptx_row_census", "ptx_comm_info", "ptx_present", "ptx_present_async", "ptx_present_poll",
            "ptx_build_info"]


class PtxConfig(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("row_begin", ctypes.c_uint32),
                ("row_end", ctypes.c_uint32), ("device", ctypes.c_int32), ("pipeline", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("reuse_radius", ctypes.c_uint32), ("reuse_neighbors", ctypes.c_uint32),
                ("temporal_cap", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 2)]


class PtxStats(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_uint64), ("kernel_ms_total", ctypes.c_double * 16),
                ("kernel_launches", ctypes.c_uint64 * 16), ("triangles", ctypes.c_uint32),
                ("bvh_nodes", ctypes.c_uint32), ("instances", ctypes.c_uint32), ("max_bvh_depth", ctypes.c_uint32),
                ("device_bytes", ctypes.c_uint64)]


class PtxError(RuntimeError):
    pass


_lib = None


def share_torch_runtime() -> None:
    """Load torch (when installed) BEFORE libptx.so so the process has ONE HIP runtime.

    torch bundles its own libamdhip64 / libhsa-runtime64 (soname .so.7 / .so.1) but links
    them by the bare name libamdhip64.so: if libptx.so loads /opt/rocm's copy first, torch
    then loads a second runtime and sees no GPU.  The other way round the dynamic linker
    hands libptx.so torch's (already loaded, same soname) runtime -- measured: same frame
    times, and torch tensors / RCCL work beside the handles (halo exchange).  Set
    PTX_STANDALONE_RUNTIME=1 to skip it."""
    if os.environ.get("PTX_STANDALONE_RUNTIME") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(path: str = LIB_PATH):
    """Load libptx.so; raises PtxError when the HIP extension is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise PtxError(f"{path} is missing: build it with `make -C pathtracerdemo_amd/csrc` "
                       "(or __graft_entry__.build()); there is no CPU fallback")
    share_torch_runtime()
    lib = ctypes.CDLL(path)
    P, H = ctypes.c_void_p, ctypes.c_void_p
    lib.ptx_abi_version.restype = ctypes.c_int
    lib.ptx_create.argtypes = [ctypes.POINTER(PtxConfig), ctypes.POINTER(H)]
    lib.ptx_upload_scene.argtypes = [H, P, ctypes.c_size_t, P, ctypes.c_size_t, P, ctypes.c_size_t]
    lib.ptx_set_frame.argtypes = [H, P]
    lib.ptx_render.argtypes = [H, P]
    lib.ptx_run_pass.argtypes = [H, ctypes.c_int]
    lib.ptx_reset_accumulation.argtypes = [H]
    lib.ptx_synchronize.argtypes = [H]
    lib.ptx_get_stats.argtypes = [H, ctypes.POINTER(PtxStats)]
    lib.ptx_reset_stats.argtypes = [H]
    lib.ptx_read_buffer.argtypes = [H, ctypes.c_int, P, ctypes.c_size_t]
    lib.ptx_write_buffer.argtypes = [H, ctypes.c_int, P, ctypes.c_size_t]
    lib.ptx_device_pointer.argtypes = [H, ctypes.c_int, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.ptx_set_stream.argtypes = [H, P]
    lib.ptx_trace.argtypes = [H, P, P, ctypes.c_size_t, ctypes.c_int]
    lib.ptx_trace_device.argtypes = [H, P, P, ctypes.c_size_t, ctypes.c_int]
    lib.ptx_present.argtypes = [H, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, P]
    lib.ptx_present_async.argtypes = [H, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
    lib.ptx_present_poll.argtypes = [H, P, ctypes.c_size_t]
    lib.ptx_build_info.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    lib.ptx_run_passes.argtypes = [H, P, ctypes.c_int]
    lib.ptx_halo_rows.argtypes = [H, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                  ctypes.POINTER(ctypes.c_size_t)]
    lib.ptx_halo_pack.argtypes = [H, P, P]
    lib.ptx_halo_unpack.argtypes = [H, P, P]
    lib.ptx_comm_unique_id.argtypes = [P, ctypes.c_size_t]
    lib.ptx_comm_init.argtypes = [H, P, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
    lib.ptx_comm_init_all.argtypes = [ctypes.POINTER(H), ctypes.c_int]
    lib.ptx_comm_info.argtypes = [H, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_uint64)]
    lib.ptx_render_bands.argtypes = [ctypes.POINTER(H), ctypes.c_int, P]
    lib.ptx_row_census.argtypes = [H, P, ctypes.c_size_t]
    lib.ptx_destroy.argtypes = [H]
    lib.ptx_last_error.argtypes = [H]
    lib.ptx_last_error.restype = ctypes.c_char_p
    for name in EXPORTED:
        if name not in ("ptx_last_error", "ptx_abi_version"):
            getattr(lib, name).restype = ctypes.c_int
    if lib.ptx_abi_version() != PTX_ABI_VERSION:
        raise PtxError(f"{path}: ABI {lib.ptx_abi_version()} != {PTX_ABI_VERSION}: rebuild it")
    _lib = lib
    return lib


def build_info(lib=None) -> dict:
    """ptx_build_info as a dict: which build this libptx.so is ("product", "ab", "wgt"), the PTX_AB
    keys it ignores, the communicator library it opened (include/ptx.h)."""
    import json
    lib = lib or load()
    buf = ctypes.create_string_buffer(2048)
    lib.ptx_build_info(buf, len(buf))
    out = json.loads(buf.value.decode())
    out["path"] = getattr(lib, "_name", LIB_PATH)
    return out


def check(lib, handle, rc: int, what: str):
    if rc != PTX_OK:
        msg = lib.ptx_last_error(handle) if handle else b""
        raise PtxError(f"{what} failed ({rc}): {msg.decode(errors='replace') if msg else ''}")
