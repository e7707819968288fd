"""Throughput of H whole-frame handles rendering concurrently (each on its own streams) vs one:
an upper-bound experiment for pipelining consecutive frames.

usage: PTX_AB=WAVE_STREAMS=2 PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so \
           python tools/concurrent_handles.py --handles 2 [--steps 20]
(WAVE_STREAMS is an A/B switch: only the measurement build, make -C pathtracerdemo_amd/csrc ab,
reads it)"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--handles", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--pipeline", default="reuse")
    ap.add_argument("--scene", default="c3_interior_32")
    a = ap.parse_args()
    from pathtracerdemo_amd.renderer import Renderer
    from pathtracerdemo_amd.scene.world import compile_scene
    cs = compile_scene(a.scene)
    rs = []
    for _ in range(a.handles):
        r = Renderer(a.width, a.height, device=0, pipeline=a.pipeline)
        r.Initialize(cs)
        rs.append(r)
    for _ in range(3):
        for r in rs:
            r.Update()
            r.Render()
    for r in rs:
        r.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        for r in rs:
            r.Update()
            r.Render()
    for r in rs:
        r.synchronize()
    dt = time.perf_counter() - t
    frames = a.steps * a.handles
    print(json.dumps({"handles": a.handles, "streams": os.environ.get("PTX_AB", ""),
                      "ms_per_frame": 1e3 * dt / frames, "msamples_s": frames * a.width * a.height / dt / 1e6}))


if __name__ == "__main__":
    main()
