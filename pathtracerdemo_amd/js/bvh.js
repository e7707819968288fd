'use strict';
/**
 * The SAH BLAS build of Mesh's constructor (GC/Structs.ts:73-80: three-mesh-bvh@0.9.2
 * computeBoundsTree({strategy: SAH, maxLeafTris: 10}), one root per geometry group) emitting
 * the library's 32-byte node records that GetBlasNode reads (SH/PT_01_GBufferPass.wgsl:310-322):
 *   w0..w5 bounds min xyz, max xyz (f32); interior: w6 = word offset of the right child from the
 *   root start (left child = node + 1), w7 = split axis; leaf: w6 = first triangle, w7 = count |
 *   0xFFFF << 16.  The index buffer is reordered so that a leaf's triangles are contiguous.
 * three-mesh-bvh is not installed here: this is the same restatement of its published SAH build
 * as the Python scene compiler's (pathtracerdemo_amd/scene/bvh.py: 32 bins, traversal cost 1,
 * triangle cost 1.25, Hoare partition, max depth 40, f32 triangle bounds as centre / half-extent
 * widened by 2^-24), step for step, so both hosts build the same trees (tests/test_node_host.py);
 * its topology against three-mesh-bvh itself stays parity-unpinned (SURVEY.md §8c).
 */
const BIN_COUNT = 32;
const TRAVERSAL_COST = 1.0;
const TRIANGLE_INTERSECT_COST = 1.25;
const FLOAT32_EPSILON = 2 ** -24;
const LEAF_FLAG = 0xFFFF0000;
const f32 = Math.fround;

/** Per triangle and axis the f32 [centre, half-extent] (computeTriangleBounds): tb[6t + 2a + {0, 1}]. */
function triangleBounds(pos, idx3, T) {
  const tb = new Float32Array(6 * T);
  for (let t = 0; t < T; t++) {
    for (let a = 0; a < 3; a++) {
      const p0 = pos[3 * idx3[3 * t] + a], p1 = pos[3 * idx3[3 * t + 1] + a], p2 = pos[3 * idx3[3 * t + 2] + a];
      const mn = Math.min(p0, p1, p2), mx = Math.max(p0, p1, p2);
      const half = (mx - mn) / 2.0;
      tb[6 * t + 2 * a] = mn + half;
      tb[6 * t + 2 * a + 1] = half + (Math.abs(mn) + half) * FLOAT32_EPSILON;
    }
  }
  return tb;
}

function surfaceArea(b) {
  const d0 = b[3] - b[0], d1 = b[4] - b[1], d2 = b[5] - b[2];
  return 2.0 * (d0 * d1 + d1 * d2 + d2 * d0);
}

class Builder {
  constructor(tb, idx3, maxLeaf, maxDepth) {
    this.tb = tb;
    this.idx3 = idx3;
    this.maxLeaf = maxLeaf;
    this.maxDepth = maxDepth;
    this.maxDepthSeen = 0;
  }

  /** node bounds and centroid bounds of triangles [lo, hi), f32 */
  bounds(lo, hi) {
    const node = [Infinity, Infinity, Infinity, -Infinity, -Infinity, -Infinity];
    const cent = [Infinity, Infinity, Infinity, -Infinity, -Infinity, -Infinity];
    const tb = this.tb;
    for (let t = lo; t < hi; t++) {
      for (let a = 0; a < 3; a++) {
        const c = tb[6 * t + 2 * a], h = tb[6 * t + 2 * a + 1];
        node[a] = Math.min(node[a], c - h);
        node[a + 3] = Math.max(node[a + 3], c + h);
        cent[a] = Math.min(cent[a], c);
        cent[a + 3] = Math.max(cent[a + 3], c);
      }
    }
    return [node.map(f32), cent.map(f32)];
  }

  split(nodeB, centB, lo, hi) {
    const count = hi - lo, tb = this.tb;
    const rootSa = surfaceArea(nodeB);
    let bestCost = TRIANGLE_INTERSECT_COST * count, axis = -1, pos = 0.0;
    const bi = new Int32Array(count);
    for (let a = 0; a < 3; a++) {
      const axisLeft = centB[a], axisLen = centB[a + 3] - axisLeft, binW = axisLen / BIN_COUNT;
      const cnt = new Float64Array(BIN_COUNT);
      const bmin = [], bmax = [];
      for (let i = 0; i < BIN_COUNT; i++) { bmin.push([Infinity, Infinity, Infinity]); bmax.push([-Infinity, -Infinity, -Infinity]); }
      for (let t = 0; t < count; t++) {
        const c = tb[6 * (lo + t) + 2 * a];
        let b = binW > 0 ? Math.floor((c - axisLeft) / binW) : 0;
        b = Math.min(Math.max(b, 0), BIN_COUNT - 1);
        bi[t] = b;
        cnt[b] += 1;
        for (let k = 0; k < 3; k++) {
          const ck = tb[6 * (lo + t) + 2 * k], hk = tb[6 * (lo + t) + 2 * k + 1];
          bmin[b][k] = Math.min(bmin[b][k], ck - hk);
          bmax[b][k] = Math.max(bmax[b][k], ck + hk);
        }
      }
      // left-to-right and right-to-left unions of the bins
      const lmin = [], lmax = [], rmin = new Array(BIN_COUNT), rmax = new Array(BIN_COUNT);
      for (let i = 0; i < BIN_COUNT; i++) {
        lmin.push(i ? bmin[i].map((v, k) => Math.min(lmin[i - 1][k], v)) : bmin[i].slice());
        lmax.push(i ? bmax[i].map((v, k) => Math.max(lmax[i - 1][k], v)) : bmax[i].slice());
      }
      for (let i = BIN_COUNT - 1; i >= 0; i--) {
        rmin[i] = i < BIN_COUNT - 1 ? bmin[i].map((v, k) => Math.min(rmin[i + 1][k], v)) : bmin[i].slice();
        rmax[i] = i < BIN_COUNT - 1 ? bmax[i].map((v, k) => Math.max(rmax[i + 1][k], v)) : bmax[i].slice();
      }
      let lcount = 0;
      for (let i = 0; i < BIN_COUNT - 1; i++) {
        lcount += cnt[i];
        const lc = lcount, rc = count - lc;
        const lp = lc && rootSa > 0 ? surfaceArea([...lmin[i], ...lmax[i]]) / rootSa : 0.0;
        const rp = rc && rootSa > 0 ? surfaceArea([...rmin[i + 1], ...rmax[i + 1]]) / rootSa : 0.0;
        const cost = TRAVERSAL_COST + TRIANGLE_INTERSECT_COST * (lp * lc + rp * rc);
        if (cost < bestCost) {
          axis = a;
          bestCost = cost;
          pos = f32(axisLeft + binW + i * binW);
        }
      }
    }
    return [axis, pos];
  }

  /** Hoare partition as three-mesh-bvh: centre < pos goes left; returns the split index. */
  partition(lo, hi, axis, pos) {
    const tb = this.tb, idx3 = this.idx3;
    const isLeft = (t) => tb[6 * t + 2 * axis] < pos;
    let nLeft = 0;
    const wrongLeft = [], wrongRight = [];
    for (let t = lo; t < hi; t++) {
      if (isLeft(t)) { nLeft++; wrongRight.push(t); } else wrongLeft.push(t);
    }
    wrongRight.reverse();
    const n = Math.min(wrongLeft.length, wrongRight.length);
    let m = 0;
    while (m < n && wrongLeft[m] < wrongRight[m]) m++;
    for (let k = 0; k < m; k++) {
      const a = wrongLeft[k], b = wrongRight[k];
      for (let q = 0; q < 6; q++) { const v = tb[6 * a + q]; tb[6 * a + q] = tb[6 * b + q]; tb[6 * b + q] = v; }
      for (let q = 0; q < 3; q++) { const v = idx3[3 * a + q]; idx3[3 * a + q] = idx3[3 * b + q]; idx3[3 * b + q] = v; }
    }
    return lo + nLeft;
  }

  build(lo, hi, nodeB, centB, depth, out) {
    this.maxDepthSeen = Math.max(this.maxDepthSeen, depth);
    const count = hi - lo, me = out.length;
    out.push(null);
    if (count <= this.maxLeaf || depth >= this.maxDepth) { out[me] = ['leaf', nodeB, lo, count]; return; }
    const [axis, pos] = this.split(nodeB, centB, lo, hi);
    if (axis === -1) { out[me] = ['leaf', nodeB, lo, count]; return; }
    const mid = this.partition(lo, hi, axis, pos);
    if (mid === lo || mid === hi) { out[me] = ['leaf', nodeB, lo, count]; return; }
    const [lb, lc] = this.bounds(lo, mid);
    this.build(lo, mid, lb, lc, depth + 1, out);
    const rightIndex = out.length;
    const [rb, rc] = this.bounds(mid, hi);
    this.build(mid, hi, rb, rc, depth + 1, out);
    out[me] = ['node', nodeB, rightIndex, axis];
  }
}

/**
 * One BVH root per [firstTriangle, triangleCount] group.  Returns {roots: Uint32Array (8 words per
 * node) per group, index: the reordered Uint32Array, maxDepth}.
 */
function buildBlas(positions, indices, groups, maxLeafTris = 10, maxDepth = 40) {
  const idx3 = Uint32Array.from(indices), T = idx3.length / 3;
  const tb = triangleBounds(positions, idx3, T);
  const b = new Builder(tb, idx3, maxLeafTris, maxDepth);
  const roots = [];
  for (const [first, count] of groups) {
    if (count === 0) throw new Error('empty sub-mesh');
    const nodes = [];
    const [nb, cb] = b.bounds(first, first + count);
    b.build(first, first + count, nb, cb, 0, nodes);
    const buf = new Uint32Array(8 * nodes.length), fv = new Float32Array(buf.buffer);
    nodes.forEach((n, i) => {
      for (let k = 0; k < 6; k++) fv[8 * i + k] = n[1][k];
      if (n[0] === 'leaf') {
        if (n[3] > 0xFFFF) throw new Error('leaf too large for the 16-bit count field');
        buf[8 * i + 6] = n[2];
        buf[8 * i + 7] = (LEAF_FLAG | n[3]) >>> 0;
      } else {
        buf[8 * i + 6] = n[2] * 8;
        buf[8 * i + 7] = n[3];
      }
    });
    roots.push(buf);
  }
  return { roots, index: idx3, maxDepth: b.maxDepthSeen };
}

module.exports = { buildBlas, triangleBounds };
