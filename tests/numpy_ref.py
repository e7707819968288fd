"""Independent pure-Python/numpy restatement of a few reference functions (test checker).

Written separately from oracle/pt_oracle.c to catch bugs the C oracle and the HIP
kernels could share.  It deliberately uses a *different* algorithm where one exists:
closest hit by brute force over every triangle (no BVH), float32 numpy arithmetic.
Cites: SH/PT_1_InitPass.wgsl (SH/ = apps/frontend/src/graphics-core/shaders/).
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def pcg(seed: int) -> int:
    """GetHashValue, SH/PT_1_InitPass.wgsl:810-815 (PCG RXS-M-XS, u32 wrap-around)."""
    state = (seed * 747796405 + 2891336453) & 0xFFFFFFFF
    word = (((state >> ((state >> 28) + 4)) ^ state) * 277803737) & 0xFFFFFFFF
    return ((word >> 22) ^ word) & 0xFFFFFFFF


def random(seed: int):
    """Random, SH/PT_1_InitPass.wgsl:817-821: f32(hash) / 4294967295.0 (== 2^32 in f32)."""
    return f32(f32(pcg(seed)) / f32(4294967295.0)), (seed + 1) & 0xFFFFFFFF


def scene_triangles_world(cs):
    """All triangles of a CompiledScene in world space: (inst, sub, prim, P0, P1, P2)."""
    S, G, U = cs.scene, cs.geometry, None
    o = cs.offsets
    out = []
    for inst in range(cs.instance_count):
        base = 33 * inst
        M = S[base:base + 16].view(np.float32).reshape(4, 4).T.astype(np.float64)
        mesh = int(S[base + 32])
        d = S[o["mesh_descriptor"] + 6 * mesh: o["mesh_descriptor"] + 6 * mesh + 6]
        off_v, off_i, _, off_root, off_b, nsub = (int(v) for v in d)
        for sub in range(nsub):
            root = int(G[o["sub_blas_root"] + off_root + sub])
            nb = o["blas"] + off_b + root
            # collect leaves of this sub-BVH
            stack = [0]
            while stack:
                n = stack.pop()
                w = cs.accel[nb + 8 * n: nb + 8 * n + 8]
                if w[7] & 0xFFFF0000:
                    first, cnt = int(w[6]), int(w[7] & 0xFFFF)
                    for prim in range(first, first + cnt):
                        ids = G[o["index"] + off_i + 3 * prim: o["index"] + off_i + 3 * prim + 3]
                        P = [G[off_v + 8 * int(v): off_v + 8 * int(v) + 3].view(np.float32) for v in ids]
                        out.append((inst, sub, prim, P, M))
                else:
                    stack += [n + 1, int(w[6]) // 8]
    return out


def brute_force_closest(tris, o, d, det_eps=1e-8):
    """Closest Moller-Trumbore hit over every triangle (local space per instance), f32."""
    best = (np.inf, None)
    for inst, sub, prim, P, M in tris:
        Minv = np.linalg.inv(M)
        lo = (Minv @ np.append(o.astype(np.float64), 1.0))[:3]
        le = (Minv @ np.append(o.astype(np.float64) + d, 1.0))[:3]
        lo, ld = lo.astype(np.float32), (le - lo).astype(np.float32)
        p0, p1, p2 = (np.asarray(p, dtype=np.float32) for p in P)
        e1, e2 = p1 - p0, p2 - p0
        pvec = np.cross(ld, e2).astype(np.float32)
        det = f32(np.dot(e1, pvec))
        if abs(det) < det_eps:
            continue
        inv = f32(1.0) / det
        tvec = lo - p0
        u = f32(np.dot(tvec, pvec)) * inv
        if u < 0 or u > 1:
            continue
        q = np.cross(tvec, e1).astype(np.float32)
        v = f32(np.dot(ld, q)) * inv
        if v < 0 or u + v > 1:
            continue
        t = f32(np.dot(e2, q)) * inv
        if t <= 1e-4:
            continue
        if t <= best[0]:
            best = (t, (inst, sub, prim))
    return best


def camera_ray(vpinv, W, H, x, y):
    """GenerateRayFromThreadID, SH/PT_01_GBufferPass.wgsl:496-507 (float64 here)."""
    M = np.asarray(vpinv, dtype=np.float32).reshape(4, 4).T.astype(np.float64)
    u = (x + 0.5) / W
    v = (y + 0.5) / H
    a = M @ np.array([2 * u - 1, 2 * v - 1, 0.0, 1.0])
    b = M @ np.array([2 * u - 1, 2 * v - 1, 1.0, 1.0])
    a, b = a[:3] / a[3], b[:3] / b[3]
    d = b - a
    return a.astype(np.float32), (d / np.linalg.norm(d)).astype(np.float32)


def ggx_d(ndoth, r):
    a = r * r
    a2 = a * a
    x = ndoth * ndoth * (a2 - 1) + 1
    return a2 / max(np.pi * x * x, 1e-4)


def brdf(n, albedo, metal, rough, v, l):
    """BRDF, SH/PT_1_InitPass.wgsl:862-889, float64."""
    n, v, l, albedo = (np.asarray(a, dtype=np.float64) for a in (n, v, l, albedo))
    h = (l + v) / np.linalg.norm(l + v)
    ndv, ndl = max(n @ v, 0), max(n @ l, 0)
    ndh, vdh = max(n @ h, 0), max(v @ h, 0)
    f0 = 0.04 * (1 - metal) + albedo * metal
    D = ggx_d(ndh, rough)
    k = (rough + 1) ** 2 / 8
    G = 1 / ((ndv * (1 - k) + k) * (ndl * (1 - k) + k))
    F = f0 + (1 - f0) * (1 - min(max(vdh, 0), 1)) ** 5
    kd = (1 - F) * (1 - metal)
    return kd / 3.141592 * albedo + F * D * G * 0.25
