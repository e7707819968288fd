"""SAH BLAS builder emitting the reference's 32-byte BVH node format.

The reference builds one BVH root per sub-mesh (glTF primitive / material group) with
three-mesh-bvh@0.9.2: ``computeBoundsTree({strategy: SAH, maxLeafTris: 10})``
(ref: apps/frontend/src/graphics-core/Structs.ts:73-80) and uploads the library's
internal ``_roots`` buffers verbatim. The WGSL reads them in ``GetBlasNode``
(ref: shaders/PT_01_GBufferPass.wgsl:310-322) and ``TraceRay`` (:540-585):

    w0..w5  bounds min xyz, max xyz (f32)
    interior: w6 = word offset of the right child from the root start (right = w6/8),
              left child = node + 1, w7 = split axis
    leaf:     w6 = first triangle (absolute within the mesh index buffer),
              w7 = count (low 16 bits) | 0xFFFF << 16

The index buffer is reordered in place so that a leaf's triangles are contiguous.
three-mesh-bvh is not available here, so this is a restatement of its published SAH
build (32 bins, traversal cost 1, triangle cost 1.25, Hoare partition, max depth 40,
f32 triangle bounds stored as centre/half-extent widened by 2^-24).  Its topology is
*parity unpinned* (SURVEY.md §8c); every consumer in this repo (oracle and HIP path)
reads the same arrays, so kernel parity does not depend on it.
"""
from __future__ import annotations

import numpy as np

BIN_COUNT = 32
TRAVERSAL_COST = 1.0
TRIANGLE_INTERSECT_COST = 1.25
FLOAT32_EPSILON = 2.0 ** -24
LEAF_FLAG = 0xFFFF0000


def _triangle_bounds(pos: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """(T,3,2) f32 [centre, half-extent] per axis, as three-mesh-bvh computeTriangleBounds."""
    tri = pos[idx.reshape(-1, 3)].astype(np.float64)            # (T,3 verts,3 axes)
    mn = tri.min(axis=1)
    mx = tri.max(axis=1)
    half = (mx - mn) / 2.0
    c = (mn + half).astype(np.float32)
    h = (half + (np.abs(mn) + half) * FLOAT32_EPSILON).astype(np.float32)
    return np.stack([c, h], axis=2)


def _surface_area(b) -> float:
    d0, d1, d2 = b[3] - b[0], b[4] - b[1], b[5] - b[2]
    return 2.0 * (d0 * d1 + d1 * d2 + d2 * d0)


class _Builder:
    def __init__(self, tb: np.ndarray, idx3: np.ndarray, max_leaf: int, max_depth: int):
        self.tb = tb            # (T,3,2) f32 centre/half
        self.idx3 = idx3        # (T,3) u32, permuted in place
        self.max_leaf = max_leaf
        self.max_depth = max_depth
        self.max_depth_seen = 0

    def bounds(self, lo: int, hi: int):
        c = self.tb[lo:hi, :, 0].astype(np.float64)
        h = self.tb[lo:hi, :, 1].astype(np.float64)
        node = np.concatenate([(c - h).min(axis=0), (c + h).max(axis=0)]).astype(np.float32)
        cent = np.concatenate([c.min(axis=0), c.max(axis=0)]).astype(np.float32)
        return node, cent

    def split(self, node_b, cent_b, lo: int, hi: int):
        count = hi - lo
        root_sa = _surface_area(node_b.astype(np.float64))
        best_cost = TRIANGLE_INTERSECT_COST * count
        axis, pos = -1, 0.0
        c_all = self.tb[lo:hi, :, 0].astype(np.float64)
        h_all = self.tb[lo:hi, :, 1].astype(np.float64)
        tmin = c_all - h_all
        tmax = c_all + h_all
        for a in range(3):
            axis_left = float(cent_b[a])
            axis_len = float(cent_b[a + 3]) - axis_left
            bin_w = axis_len / BIN_COUNT
            cand = axis_left + bin_w + np.arange(BIN_COUNT) * bin_w
            if bin_w > 0:
                bi = np.floor((c_all[:, a] - axis_left) / bin_w).astype(np.int64)
            else:
                bi = np.zeros(count, dtype=np.int64)
            bi = np.clip(bi, 0, BIN_COUNT - 1)
            cnt = np.bincount(bi, minlength=BIN_COUNT)
            bmin = np.full((BIN_COUNT, 3), np.inf)
            bmax = np.full((BIN_COUNT, 3), -np.inf)
            np.minimum.at(bmin, bi, tmin)
            np.maximum.at(bmax, bi, tmax)
            # right-to-left cache of unions
            rmin = np.minimum.accumulate(bmin[::-1], axis=0)[::-1]
            rmax = np.maximum.accumulate(bmax[::-1], axis=0)[::-1]
            lmin = np.minimum.accumulate(bmin, axis=0)
            lmax = np.maximum.accumulate(bmax, axis=0)
            lcount = np.cumsum(cnt)
            for i in range(BIN_COUNT - 1):
                lc = int(lcount[i])
                rc = count - lc
                lp = _surface_area(np.concatenate([lmin[i], lmax[i]])) / root_sa if lc and root_sa > 0 else 0.0
                rp = _surface_area(np.concatenate([rmin[i + 1], rmax[i + 1]])) / root_sa if rc and root_sa > 0 else 0.0
                cost = TRAVERSAL_COST + TRIANGLE_INTERSECT_COST * (lp * lc + rp * rc)
                if cost < best_cost:
                    axis, best_cost, pos = a, cost, float(np.float32(cand[i]))
        return axis, pos

    def partition(self, lo: int, hi: int, axis: int, pos: float) -> int:
        """Hoare partition exactly as three-mesh-bvh: centre < pos goes left."""
        c = self.tb[lo:hi, axis, 0].astype(np.float64)
        is_left = c < pos
        n_left = int(np.count_nonzero(is_left))
        wrong_left = np.nonzero(~is_left)[0]
        wrong_right = np.nonzero(is_left)[0][::-1]
        n = min(len(wrong_left), len(wrong_right))
        m = int(np.count_nonzero(wrong_left[:n] < wrong_right[:n]))
        if m:
            a = lo + wrong_left[:m]
            b = lo + wrong_right[:m]
            self.tb[a], self.tb[b] = self.tb[b].copy(), self.tb[a].copy()
            self.idx3[a], self.idx3[b] = self.idx3[b].copy(), self.idx3[a].copy()
        return lo + n_left

    def build(self, lo: int, hi: int, node_b, cent_b, depth: int, out: list):
        self.max_depth_seen = max(self.max_depth_seen, depth)
        count = hi - lo
        me = len(out)
        out.append(None)
        if count <= self.max_leaf or depth >= self.max_depth:
            out[me] = ("leaf", node_b, lo, count)
            return
        axis, pos = self.split(node_b, cent_b, lo, hi)
        if axis == -1:
            out[me] = ("leaf", node_b, lo, count)
            return
        mid = self.partition(lo, hi, axis, pos)
        if mid == lo or mid == hi:
            out[me] = ("leaf", node_b, lo, count)
            return
        lb, lc = self.bounds(lo, mid)
        self.build(lo, mid, lb, lc, depth + 1, out)
        right_index = len(out)
        rb, rc = self.bounds(mid, hi)
        self.build(mid, hi, rb, rc, depth + 1, out)
        out[me] = ("node", node_b, right_index, axis)


def build_blas(positions: np.ndarray, indices: np.ndarray, groups: list[tuple[int, int]],
               max_leaf_tris: int = 10, max_depth: int = 40):
    """Build one BVH root per (first_tri, tri_count) group.

    Returns (roots: list[np.ndarray u32 (8*nodes,)], reordered indices (u32), max depth).
    """
    idx3 = indices.reshape(-1, 3).copy()
    tb = _triangle_bounds(positions, idx3.reshape(-1))
    b = _Builder(tb, idx3, max_leaf_tris, max_depth)
    roots = []
    for first, count in groups:
        if count == 0:
            raise ValueError("empty sub-mesh")
        nodes: list = []
        nb, cb = b.bounds(first, first + count)
        b.build(first, first + count, nb, cb, 0, nodes)
        buf = np.zeros((len(nodes), 8), dtype=np.uint32)
        fview = buf.view(np.float32)
        for i, n in enumerate(nodes):
            fview[i, 0:6] = n[1]
            if n[0] == "leaf":
                if n[3] > 0xFFFF:
                    raise ValueError("leaf too large for the 16-bit count field")
                buf[i, 6] = n[2]
                buf[i, 7] = LEAF_FLAG | n[3]
            else:
                buf[i, 6] = n[2] * 8
                buf[i, 7] = n[3]
        roots.append(buf.reshape(-1))
    return roots, idx3.reshape(-1).astype(np.uint32), b.max_depth_seen
