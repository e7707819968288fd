"""Capture the straggler queries of trace_queue (diagnostic build): every trace call that ran
>= kStragglerAabb slab tests (ptx_device.h) over one frame, with its ray, bound and result.

usage (GPU box):  make -C pathtracerdemo_amd/csrc wgt
                  PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so \\
                      python tools/stragglers.py --out gpurun_out/stragglers.npz
The .npz holds o, d, t_max, slab tests, triangle tests, hit t / instance / sub-mesh / prim per
straggler; the printout is their count and slab-test distribution by query kind (closest hit:
t_max = 1e10; Visibility: the light distance)."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KID_STRAGGLER, KID_STRAGGLER2 = 13, 14


def lo32f(a):
    return (a & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32)


def hi32f(a):
    return (a >> np.uint64(32)).astype(np.uint32).view(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--pipeline", default="reuse")
    ap.add_argument("--scene", default="c3_interior_32")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from pathtracerdemo_amd import _native as N
    from pathtracerdemo_amd.renderer import Renderer
    from pathtracerdemo_amd.scene.world import compile_scene
    lib = N.load()
    lib.ptx_diag_wave_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.ptx_diag_wave_times.restype = ctypes.c_int
    r = Renderer(a.width, a.height, device=0, pipeline=a.pipeline, single_stream=True, time_launches=True)
    r.Initialize(compile_scene(a.scene))
    buf = np.zeros((1 << 20, 4), dtype=np.uint64)
    for _ in range(2):
        r.Update()
        r.Render()
    r.synchronize()
    lib.ptx_diag_wave_times(r._h, buf.ctypes.data, 1 << 20)
    r.Update()
    r.Render()
    r.synchronize()
    n = lib.ptx_diag_wave_times(r._h, buf.ctypes.data, 1 << 20)
    r.close()
    rec = buf[:n]
    kid = (rec[:, 2] >> np.uint64(32)).astype(np.int64) & 0x7F
    A = np.nonzero(kid == KID_STRAGGLER)[0]
    A = A[A + 1 < n]
    A = A[kid[A + 1] == KID_STRAGGLER2]
    ra, rb = rec[A], rec[A + 1]
    o = np.stack([lo32f(ra[:, 0]), hi32f(ra[:, 0]), lo32f(ra[:, 1])], 1)
    d = np.stack([hi32f(ra[:, 1]), lo32f(rb[:, 0]), hi32f(rb[:, 0])], 1)
    aabb = (ra[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    tri = (ra[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    tmax = hi32f(ra[:, 3])
    t = lo32f(rb[:, 1])
    inst = (rb[:, 1] >> np.uint64(32)).astype(np.int64)
    prim = (rb[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    sub = rb[:, 3].astype(np.int64)
    vis = tmax < 1e10
    print(f"{len(A)} straggler trace calls (>= 256 slab tests) in one {a.width}x{a.height} {a.pipeline} frame")
    for name, m in (("closest", ~vis), ("visibility", vis)):
        if m.any():
            q = np.percentile(aabb[m], [50, 90, 99, 100])
            print(f"  {name:10s} {m.sum():7d}  slab tests p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} max {q[3]:.0f}"
                  f"  tri tests p50 {np.percentile(tri[m], 50):.0f} max {tri[m].max()}")
    edges = [256, 512, 1024, 2048, 4096, 8192, 1 << 30]
    h = np.histogram(aabb, bins=edges)[0]
    print("  slab-test histogram: " + ", ".join(f"[{edges[i]},{edges[i+1]}): {h[i]}" for i in range(len(h))))
    # hit surfaces of the worst ones
    worst = np.argsort(-aabb)[:20]
    for k in worst:
        print(f"  aabb {aabb[k]:6d} tri {tri[k]:5d} o ({o[k,0]:+.4f},{o[k,1]:+.4f},{o[k,2]:+.4f}) d ({d[k,0]:+.4f},"
              f"{d[k,1]:+.4f},{d[k,2]:+.4f}) t_max {tmax[k]:.4g} hit t {t[k]:.4g} inst {inst[k]} sub {sub[k]} prim {prim[k]}")
    if a.out:
        np.savez(a.out, o=o, d=d, t_max=tmax, aabb=aabb, tri=tri, t=t, inst=inst, sub=sub, prim=prim)


if __name__ == "__main__":
    main()
