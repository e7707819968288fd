"""Band handles exchanging their halos through ptx_comm.cpp's RCCL code, in ONE process on ONE
GPU, over the loopback communicator (tests/loopback/loopback_rccl.cpp).  Run by
tests/test_gpu_loopback.py as a child process with PTX_RCCL_LIB set (libptx.so loads the RCCL
library once per process); prints one JSON object with what it measured.

Each band handle owns a communicator (ptx_comm_init, the neighbour check) made from its own
host thread, as the ranks of a multi-GPU job are separate processes; frames are rendered by one
thread per band (ptx_render -> render_band_nccl: grouped send / recv of the static halo, the
motion halo on moved frames, pipelined frames) or by ptx_render_bands from one thread (its
communicator branch).  Every frame is compared with one handle of the whole image.
"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pathtracerdemo_amd.renderer import Renderer  # noqa: E402
from pathtracerdemo_amd.scene.world import compile_scene  # noqa: E402

# tests/test_gpu_reuse.py's interactive path, then a fast pitch turn past the motion halo
PATH = [((0.0, 0.0, 6.0), 0.0, 0.0), ((0.083, 0.0, 6.0), 0.0, 0.0), ((0.166, 0.0, 5.95), 0.0, 0.0),
        ((0.25, 0.02, 5.9), 1.5, 0.0), ((0.25, 0.02, 5.9), 3.0, 0.0), ((0.2, 0.02, 5.85), 4.5, 0.0),
        ((0.2, 0.02, 5.85), 4.5, 0.0), ((0.12, 0.0, 5.8), 3.0, 0.0), ((0.12, 0.0, 5.8), 3.0, 12.0),
        ((0.12, 0.0, 5.8), 3.0, 12.0)]


def run_threads(fns):
    errs = [None] * len(fns)

    def wrap(i, f):
        try:
            f()
        except Exception as e:  # noqa: BLE001 -- reported to the parent
            errs[i] = f"{type(e).__name__}: {e}"

    ts = [threading.Thread(target=wrap, args=(i, f)) for i, f in enumerate(fns)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    if any(t.is_alive() for t in ts):
        raise SystemExit("a band thread did not finish within 120 s")
    return errs


def pose(r, loc, yaw, pitch):
    c = r.GetCamera()
    c.set_location(*loc)
    c.set_yaw(yaw)
    c.set_pitch(pitch)
    r.Update()


def differs(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype != np.uint32:
        a, b = a.view(np.uint32), b.view(np.uint32)
    return int(np.any(a != b, axis=-1).sum())


def make(cs, W, H, R, a=0, b=0, pipeline="reuse"):
    r = Renderer(W, H, device=0, pipeline=pipeline, reuse_radius=R, row_begin=a, row_end=b)
    r.Initialize(cs)
    return r


def connect(bands):
    uid = Renderer.comm_unique_id()
    errs = run_threads([lambda r=r, k=k: r.comm_init(uid, k, len(bands)) for k, r in enumerate(bands)])
    assert not any(errs), errs


def compare(one, bands):
    return {"history": differs(np.concatenate([b.read_history() for b in bands]), one.read_history()),
            "temporal": differs(np.concatenate([b.read_reservoir() for b in bands]), one.read_reservoir()),
            "radiance": differs(np.concatenate([b.read_image() for b in bands]), one.read_image())}


def scenario_split(cs, out):
    """4 bands (R = 12) along PATH, one thread per band, then ptx_render_bands from one thread."""
    W, H, R = 96, 128, 12
    cuts = [0, 30, 64, 100, 128]
    one = make(cs, W, H, R)
    bands = [make(cs, W, H, R, a, b) for a, b in zip(cuts, cuts[1:])]
    connect(bands)
    frames = []
    for f, (loc, yaw, pitch) in enumerate(PATH, start=1):
        pose(one, loc, yaw, pitch)
        one.Render()
        for b in bands:
            pose(b, loc, yaw, pitch)
        errs = run_threads([b.Render for b in bands])
        assert not any(errs), errs
        frames.append({"frame": f, **compare(one, bands)})
    for f, (loc, yaw, pitch) in enumerate([((0.1, 0.05, 5.7), 2.0, 6.0), ((0.1, 0.05, 5.7), 2.0, 6.0),
                                           ((0.0, 0.0, 5.9), 0.0, 0.0)], start=len(PATH) + 1):
        pose(one, loc, yaw, pitch)
        one.Render()
        for b in bands:
            pose(b, loc, yaw, pitch)
        Renderer.render_bands(bands)
        frames.append({"frame": f, "render_bands": True, **compare(one, bands)})
    out["split"] = {"frames": frames,
                    "clips_bands": int(sum(b.read_counters()["motion_clips"] for b in bands)),
                    "clips_one": int(one.read_counters()["motion_clips"]),
                    "hist_used": float((one.read_reservoir()[..., 29] > 1).mean()),
                    "comm": [b.comm_info() for b in bands]}
    for r in [one] + bands:
        r.close()


def scenario_gi_split(cs, out):
    """ReSTIR GI as 3 communicator bands (R = 8) along PATH: the GI motion pass reads the motion
    halo (previous spatial output) and the previous static halo (G-buffer rows)."""
    W, H, R = 64, 96, 8
    cuts = [0, 40, 70, 96]
    one = make(cs, W, H, R, pipeline="gi")
    bands = [make(cs, W, H, R, a, b, pipeline="gi") for a, b in zip(cuts, cuts[1:])]
    connect(bands)
    frames = []
    for f, (loc, yaw, pitch) in enumerate(PATH, start=1):
        pose(one, loc, yaw, pitch)
        one.Render()
        for b in bands:
            pose(b, loc, yaw, pitch)
        errs = run_threads([b.Render for b in bands])
        assert not any(errs), errs
        frames.append({"frame": f, **compare(one, bands)})
    out["gi_split"] = {"frames": frames,
                       "clips_bands": int(sum(b.read_counters()["motion_clips"] for b in bands)),
                       "clips_one": int(one.read_counters()["motion_clips"]),
                       "hist_used": float((one.read_reservoir()[..., 11] > 1).mean())}
    for r in [one] + bands:
        r.close()


def scenario_reset_one_rank(cs, out):
    """one rank drops its history (reset) while the camera moves; the ranks still agree
    on the motion halo (decided from the uniform sequence) and both frames complete."""
    W, H, R = 64, 64, 8
    bands = [make(cs, W, H, R, 0, 32), make(cs, W, H, R, 32, 64)]
    connect(bands)
    t0 = time.time()
    res = []
    for f, (loc, yaw, pitch) in enumerate(PATH[:5], start=1):
        if f == 3:
            bands[1].reset_accumulation()
        for b in bands:
            pose(b, loc, yaw, pitch)
        errs = run_threads([b.Render for b in bands])
        res.append(errs)
        for b in bands:
            b.synchronize()
    out["reset_one_rank"] = {"errors": res, "seconds": round(time.time() - t0, 2),
                             "finite": bool(all(np.isfinite(b.read_image()).all() for b in bands))}
    for b in bands:
        b.close()


def scenario_dead_peer(cs, out, stats):
    """A rank whose peer never renders: its frame fails with an error status after the deadline
    (no hang), and its communicator is then aborted, not destroyed."""
    W, H, R = 64, 64, 8
    bands = [make(cs, W, H, R, 0, 32), make(cs, W, H, R, 32, 64)]
    connect(bands)
    before = stats()
    pose(bands[0], (0.0, 0.0, 6.0), 0.0, 0.0)
    t0 = time.time()
    err = None
    try:
        bands[0].Render()
        bands[0].synchronize()
    except Exception as e:  # noqa: BLE001
        err = str(e)
    took = time.time() - t0
    bands[0].close()
    mid = stats()
    bands[1].close()
    after = stats()
    out["dead_peer"] = {"error": err, "seconds": round(took, 2), "aborts": mid[4] - before[4],
                        "destroys_healthy": after[3] - mid[3], "finalizes_healthy": after[5] - mid[5]}


def main():
    lib = ctypes.CDLL(os.environ["PTX_RCCL_LIB"])
    buf = (ctypes.c_ulonglong * 6)()

    def stats():
        lib.loopback_stats(buf)
        return list(buf)

    cs = compile_scene("c3_interior_32")
    out = {}
    scenario_split(cs, out)
    scenario_gi_split(cs, out)
    scenario_reset_one_rank(cs, out)
    scenario_dead_peer(cs, out, stats)
    out["stub"] = dict(zip(["groups", "pairs", "bytes", "destroys", "aborts", "finalizes"], stats()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
