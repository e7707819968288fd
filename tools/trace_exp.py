#!/usr/bin/env python3
"""Traversal-throughput experiment: Grays/s of ptx_trace on ray sets of varying coherence.

Run on the GPU box:  python tools/trace_exp.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import uniform_for  # noqa: E402
from pathtracerdemo_amd import _native as N  # noqa: E402
from pathtracerdemo_amd.renderer import Renderer  # noqa: E402
from pathtracerdemo_amd.scene.world import compile_scene  # noqa: E402


def primary_rays(u, W, H, order="tile"):
    m = u[4:20].view(np.float32).reshape(4, 4).T.astype(np.float64)
    ys, xs = np.mgrid[0:H, 0:W]
    if order == "tile":
        tx, ty = xs // 8, ys // 8
        key = (ty * ((W + 7) // 8) + tx) * 64 + (ys % 8) * 8 + (xs % 8)
        idx = np.argsort(key.reshape(-1), kind="stable")
    else:
        idx = np.random.default_rng(0).permutation(W * H)
    xs, ys = xs.reshape(-1)[idx], ys.reshape(-1)[idx]
    u_ = (xs + 0.5) / W * 2 - 1
    v_ = (ys + 0.5) / H * 2 - 1
    a = np.stack([u_, v_, np.zeros_like(u_), np.ones_like(u_)], 1) @ m.T
    b = np.stack([u_, v_, np.ones_like(u_), np.ones_like(u_)], 1) @ m.T
    a = a[:, :3] / a[:, 3:]
    b = b[:, :3] / b[:, 3:]
    d = b - a
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((len(a), 8), np.float32)
    r[:, 0:3] = a
    r[:, 3:6] = d
    return r


def timed(r, rays, mode, reps=5):
    hits = r.trace(rays, mode)  # warm + staging alloc
    r.reset_stats()
    for _ in range(reps):
        r.trace(rays, mode)
    st = r.stats()
    ms = st["kernel_ms_total"][N.PTX_PASS_TRACE] / st["kernel_launches"][N.PTX_PASS_TRACE]
    return ms, hits


def main():
    W, H = 1920, 1080
    cs = compile_scene("dummy_scene_1")
    r = Renderer(W, H, device=0)
    r.Initialize(cs)
    u = uniform_for(cs, W, H)
    r.set_uniform(u)
    out = {}
    prim = primary_rays(u, W, H, "tile")
    ms, hits = timed(r, prim, 0)
    out["primary_tile"] = ms
    ms, _ = timed(r, primary_rays(u, W, H, "random"), 0)
    out["primary_random_order"] = ms
    valid = (hits[:, 1].view(np.uint32) >> 31) == 1
    pos = hits[valid, 5:8]
    n = len(pos)
    rng = np.random.default_rng(1)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    bounce = np.zeros((n, 8), np.float32)
    bounce[:, 0:3] = pos
    bounce[:, 3:6] = d
    out["bounce_pixel_order"], _ = timed(r, bounce, 1)
    octant = (d[:, 0] < 0) * 1 + (d[:, 1] < 0) * 2 + (d[:, 2] < 0) * 4
    out["bounce_octant_sorted"], _ = timed(r, bounce[np.argsort(octant, kind="stable")], 1)
    lights = np.array([[0, 0, 1e11], [0, 0, -1], [0, 1, -2]], np.float64)  # sun(-dir*INF), point, rect centre

    def shadow(lid):
        tgt = lights[lid] if lid.ndim == 0 else lights[lid]
        v = tgt - pos.astype(np.float64)
        dist = np.linalg.norm(v, axis=1, keepdims=True)
        s = np.zeros((n, 8), np.float32)
        s[:, 0:3] = pos
        s[:, 3:6] = v / dist
        return s
    out["shadow_point_light"], _ = timed(r, shadow(np.ones(n, int)), 1)
    lid = rng.integers(0, 3, size=n)
    sr = shadow(lid)
    out["shadow_random_light"], _ = timed(r, sr, 1)
    out["shadow_random_light_sorted"], _ = timed(r, sr[np.argsort(lid, kind="stable")], 1)
    res = {k: {"ms": round(v, 4), "Mrays": n if not k.startswith("primary") else W * H} for k, v in out.items()}
    for k, v in res.items():
        v["Grays_s"] = round(v["Mrays"] / v["ms"] / 1e6, 3)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
