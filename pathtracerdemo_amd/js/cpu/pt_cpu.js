'use strict';
/**
 * pt_cpu.js -- the reference's live per-pixel path (PT_01 G-buffer -> PT_1 init -> PT_4
 * final) restated in JavaScript for the CPU baseline of SURVEY.md §8(d) ("the same JS CPU
 * tracer ... on the node's host cores, worker_threads").  It runs on the reference's own
 * device arrays (uniform block, SceneBuffer, GeometryBuffer, AccelBuffer; Renderer_TEST.ts
 * :165-206, :267-420) and follows the WGSL function by function (SH/ =
 * apps/frontend/src/graphics-core/shaders/): TraceRay over the three-mesh-bvh BLAS
 * (PT_1:605-715), GetSurface (:438-467), BSDF / sampling / PDFs (:834-1245), SampleNEE
 * (:970-1025), Visibility (:774-802), the init path tree (:1361-1486), RegeneratePath +
 * PathContribution (PT_4:1306-1428).
 *
 * Every f32 operation is rounded with Math.fround, in the operation order DESIGN.md
 * §Numerics fixes (double rounding is exact for + - * / sqrt of f32 operands), with the
 * same fixed sin/cos/pow5 as the C oracle -- so its buffers are bit-identical to the
 * oracle's (tests/test_js_cpu.py).  A baseline, not a product path.
 */
const f = Math.fround;

// constants, SH/PT_1_InitPass.wgsl:193-221
const STRIDE_INSTANCE = 33, STRIDE_LIGHT = 18, STRIDE_DESCRIPTOR = 6, STRIDE_MATERIAL = 15, STRIDE_VERTEX = 8;
const STRIDE_BLAS = 8;
const RECONNECTION_DISTANCE = f(0.1), RECONNECTION_ROUGHNESS = f(0.5);
const INF_F = f(1e11), EPS_F = f(1e-4), PI_F = f(3.141592), ENV_C = f(0.5);
const LIGHT_DIRECTION = 0, LIGHT_POINT = 1, LIGHT_RECT = 2, LIGHT_ENV = 3;
const LOBE_LAMBERT = 0, LOBE_GGX = 1, LOBE_LIGHT = 3;
const U_W = 0, U_H = 1, U_VPINV = 4, U_FRAME = 23, U_OFF_DESC = 24, U_OFF_MAT = 25, U_OFF_LIGHT = 26,
  U_OFF_CDF = 27, U_OFF_INDEX = 28, U_OFF_SUBROOT = 29, U_OFF_BLAS = 30, U_INST_COUNT = 31, U_LIGHT_COUNT = 32;
const EPS_GBUFFER = { det: f(1e-8), bary: f(1e-6), final: false };
const EPS_INIT = { det: f(1e-4), bary: f(1e-8), final: false };
const EPS_FINAL = { det: f(1e-4), bary: f(1e-8), final: true };

// ---------------------------------------------------------------- f32 vector algebra
const V3 = (x, y, z) => ({ x, y, z });
const vadd = (a, b) => V3(f(a.x + b.x), f(a.y + b.y), f(a.z + b.z));
const vsub = (a, b) => V3(f(a.x - b.x), f(a.y - b.y), f(a.z - b.z));
const vmul = (a, b) => V3(f(a.x * b.x), f(a.y * b.y), f(a.z * b.z));
const vscale = (a, s) => V3(f(a.x * s), f(a.y * s), f(a.z * s));
const vdivs = (a, s) => V3(f(a.x / s), f(a.y / s), f(a.z / s));
const vneg = (a) => V3(-a.x, -a.y, -a.z);
const vdot = (a, b) => f(f(f(a.x * b.x) + f(a.y * b.y)) + f(a.z * b.z));
const vcross = (a, b) => V3(f(f(a.y * b.z) - f(a.z * b.y)), f(f(a.z * b.x) - f(a.x * b.z)), f(f(a.x * b.y) - f(a.y * b.x)));
const vlength = (a) => f(Math.sqrt(vdot(a, a)));
const vnormalize = (a) => vdivs(a, vlength(a));
// C fminf / fmaxf: a NaN operand yields the other one; ties return the second operand
const fmin = (a, b) => (a !== a ? b : b !== b ? a : a < b ? a : b);
const fmax = (a, b) => (a !== a ? b : b !== b ? a : a > b ? a : b);
const saturate = (a) => fmin(fmax(a, 0), 1);
const mixf = (a, b, t) => f(f(a * f(1 - t)) + f(b * t));
const vmix = (a, b, t) => V3(mixf(a.x, b.x, t), mixf(a.y, b.y, t), mixf(a.z, b.z, t));
const L_R = f(0.2126), L_G = f(0.7152), L_B = f(0.0722);
const luminance = (c) => f(f(f(c.x * L_R) + f(c.y * L_G)) + f(c.z * L_B));

// column-major mat4 (m[off + 4*col + row]) * vec4(p, 1), then /w (SH/PT_1_InitPass.wgsl:480-484)
function xformPoint(m, o, p) {
  const x = f(f(f(f(m[o] * p.x) + f(m[o + 4] * p.y)) + f(m[o + 8] * p.z)) + m[o + 12]);
  const y = f(f(f(f(m[o + 1] * p.x) + f(m[o + 5] * p.y)) + f(m[o + 9] * p.z)) + m[o + 13]);
  const z = f(f(f(f(m[o + 2] * p.x) + f(m[o + 6] * p.y)) + f(m[o + 10] * p.z)) + m[o + 14]);
  const w = f(f(f(f(m[o + 3] * p.x) + f(m[o + 7] * p.y)) + f(m[o + 11] * p.z)) + m[o + 15]);
  return V3(f(x / w), f(y / w), f(z / w));
}
// transpose(m) * vec4(p, 1), then /w (normal transform, SH/PT_1_InitPass.wgsl:395)
function xformPointT(m, o, p) {
  const x = f(f(f(f(m[o] * p.x) + f(m[o + 1] * p.y)) + f(m[o + 2] * p.z)) + m[o + 3]);
  const y = f(f(f(f(m[o + 4] * p.x) + f(m[o + 5] * p.y)) + f(m[o + 6] * p.z)) + m[o + 7]);
  const z = f(f(f(f(m[o + 8] * p.x) + f(m[o + 9] * p.y)) + f(m[o + 10] * p.z)) + m[o + 11]);
  const w = f(f(f(f(m[o + 12] * p.x) + f(m[o + 13] * p.y)) + f(m[o + 14] * p.z)) + m[o + 15]);
  return V3(f(x / w), f(y / w), f(z / w));
}

// ---------------------------------------------------------------- RNG, PT_1:810-826
function pcg(seed) {
  const state = (Math.imul(seed, 747796405) + 2891336453) >>> 0;
  const word = Math.imul(((state >>> ((state >>> 28) + 4)) ^ state) >>> 0, 277803737) >>> 0;
  return ((word >>> 22) ^ word) >>> 0;
}
const R_SCALE = f(4294967295); // the WGSL literal rounds to 2^32 in f32
function random(st) { // st = {s}: Random() then seed++
  const h = pcg(st.s);
  st.s = (st.s + 1) >>> 0;
  return f(f(h) / R_SCALE);
}

// ---------------------------------------------------------------- fixed transcendentals (= oracle pow5_/sincos_)
const pow5 = (x) => { const x2 = f(x * x); return f(f(x2 * x2) * x); };
const SC = [f(1.27323954473516), f(0.78515625), f(2.4187564849853515625e-4), f(3.77489497744594108e-8),
  f(-1.9515295891e-4), f(8.3321608736e-3), f(1.6666654611e-1), f(2.443315711809948e-5),
  f(1.388731625493765e-3), f(4.166664568298827e-2)];
function sincos(x) {
  let j = Math.trunc(f(x * SC[0]));
  let y = f(j);
  if (j & 1) { j += 1; y = f(y + 1); }
  j &= 7;
  const z = f(f(f(x - f(y * SC[1])) - f(y * SC[2])) - f(y * SC[3]));
  const zz = f(z * z);
  const ps = f(f(f(f(f(f(f(SC[4] * zz) + SC[5]) * zz) - SC[6]) * zz) * z) + z);
  const a4 = f(f(f(f(SC[7] * zz) - SC[8]) * zz) + SC[9]);
  const pc = f(f(f(f(a4 * zz) * zz) - f(f(0.5) * zz)) + 1);
  if (j === 0) return [ps, pc];
  if (j === 2) return [pc, -ps];
  if (j === 4) return [-ps, -pc];
  return [-pc, ps];
}

class CpuTracer {
  /** uniform: Uint32Array(33); scene, geometry, accel: Uint32Array (SerializeWorldData). */
  constructor(uniform, scene, geometry, accel) {
    this.U = uniform;
    this.S = scene; this.Sf = new Float32Array(scene.buffer, scene.byteOffset, scene.length);
    this.G = geometry; this.Gf = new Float32Array(geometry.buffer, geometry.byteOffset, geometry.length);
    this.A = accel; this.Af = new Float32Array(accel.buffer, accel.byteOffset, accel.length);
    this.W = uniform[U_W]; this.H = uniform[U_H];
    this.eps = EPS_INIT;
    this.stack = new Uint32Array(96);
  }

  // ------------------------------------------------------------ scene access
  desc(mesh) { const o = this.U[U_OFF_DESC] + STRIDE_DESCRIPTOR * mesh, S = this.S; return { vtx: S[o], idx: S[o + 1], mat: S[o + 2], root: S[o + 3], blas: S[o + 4], nsub: S[o + 5] }; }
  instMesh(i) { return this.S[STRIDE_INSTANCE * i + 32]; }
  material(d, mid) { // GetMaterial, PT_1:285-314
    const o = this.U[U_OFF_MAT] + d.mat + STRIDE_MATERIAL * mid, F = this.Sf;
    const m = { albedo: V3(F[o], F[o + 1], F[o + 2]), metal: F[o + 8], rough: F[o + 9], trans: F[o + 10], ior: F[o + 11] };
    if (m.trans > 0) m.albedo = V3(1, 1, 0);
    m.rough = fmax(m.rough, f(0.01));
    return m;
  }
  vpos(d, v) { const o = d.vtx + STRIDE_VERTEX * v, F = this.Gf; return V3(F[o], F[o + 1], F[o + 2]); }
  vnrm(d, v) { const o = d.vtx + STRIDE_VERTEX * v, F = this.Gf; return V3(F[o + 3], F[o + 4], F[o + 5]); }
  triIds(d, prim) { const o = this.U[U_OFF_INDEX] + d.idx + 3 * prim, G = this.G; return [G[o], G[o + 1], G[o + 2]]; }
  blasNode(d, sub, node) { // GetBlasNode, PT_01:310-322 -> word offset into A
    return this.U[U_OFF_BLAS] + d.blas + this.G[this.U[U_OFF_SUBROOT] + d.root + sub] + STRIDE_BLAS * node;
  }
  surface(x) { // GetSurface, PT_1:438-467
    const d = this.desc(this.instMesh(x.inst)), F = this.Sf;
    const mo = STRIDE_INSTANCE * x.inst, io = mo + 16;
    const mat = this.material(d, x.mat);
    const id = this.triIds(d, x.prim);
    const p0 = xformPoint(F, mo, this.vpos(d, id[0])), n0 = xformPointT(F, io, this.vnrm(d, id[0]));
    const p1 = xformPoint(F, mo, this.vpos(d, id[1])), n1 = xformPointT(F, io, this.vnrm(d, id[1]));
    const p2 = xformPoint(F, mo, this.vpos(d, id[2])), n2 = xformPointT(F, io, this.vnrm(d, id[2]));
    const U = x.bu, V = x.bv, W = f(f(1 - U) - V);
    return {
      nrm: vnormalize(vadd(vadd(vscale(n0, U), vscale(n1, V)), vscale(n2, W))),
      pos: vadd(vadd(vscale(p0, U), vscale(p1, V)), vscale(p2, W)), mat,
    };
  }

  // ------------------------------------------------------------ traversal
  aabbRange(r, inv, o) { // GetRayAABBIntersectionRange, PT_1:498-514 -> [tmin, tmax]
    const F = this.Af;
    const t1x = f(f(F[o] - r.o.x) * inv.x), t1y = f(f(F[o + 1] - r.o.y) * inv.y), t1z = f(f(F[o + 2] - r.o.z) * inv.z);
    const t2x = f(f(F[o + 3] - r.o.x) * inv.x), t2y = f(f(F[o + 4] - r.o.y) * inv.y), t2z = f(f(F[o + 5] - r.o.z) * inv.z);
    const tmin = fmax(fmin(t1x, t2x), fmax(fmin(t1y, t2y), fmin(t1z, t2z)));
    const tmax = fmin(fmax(t1x, t2x), fmin(fmax(t1y, t2y), fmax(t1z, t2z)));
    return tmin > tmax ? [1, 0] : [tmin, tmax];
  }
  rayTri(r, P0, P1, P2) { // GetRayTriangleHitDistance, PT_1:516-547
    const e1 = vsub(P1, P0), e2 = vsub(P2, P0);
    const pvec = vcross(r.d, e2);
    const det = vdot(e1, pvec);
    if (Math.abs(det) < this.eps.det) return INF_F;
    const inv = f(1 / det);
    const tvec = vsub(r.o, P0);
    const u = f(vdot(tvec, pvec) * inv);
    if (u < 0 || u > 1) return INF_F;
    const qvec = vcross(tvec, e1);
    const v = f(vdot(r.d, qvec) * inv);
    if (v < 0 || f(u + v) > 1) return INF_F;
    const t = f(vdot(e2, qvec) * inv);
    if (t <= f(1e-4)) return INF_F;
    return t;
  }
  trace(ray) { // TraceRay, PT_1:605-715 (PT_01:509-621 identical up to epsilons)
    const vx = f(1e-4);
    let vy = f(1e10), valid = false, binst = 0, bsub = 0, bprim = 0;
    const A = this.A, stack = this.stack, F = this.Sf, ninst = this.U[U_INST_COUNT];
    for (let inst = 0; inst < ninst; ++inst) {
      const d = this.desc(this.instMesh(inst));
      const io = STRIDE_INSTANCE * inst + 16;
      const start = xformPoint(F, io, ray.o), end = xformPoint(F, io, vadd(ray.o, ray.d));
      const local = { o: start, d: vsub(end, start) };
      const inv = V3(f(1 / local.d.x), f(1 / local.d.y), f(1 / local.d.z));
      for (let sub = 0; sub < d.nsub; ++sub) {
        let rr = this.aabbRange(local, inv, this.blasNode(d, sub, 0));
        if (!(vx <= rr[1] && rr[0] <= vy)) continue;
        let sp = 0;
        stack[0] = 0;
        while (sp > 0 || sp === 0) {
          const id = stack[sp--];
          const node = this.blasNode(d, sub, id);
          if ((A[node + 7] & 0xffff0000) === 0) {
            const lid = id + 1, rid = A[node + 6] >>> 3;
            const l = this.aabbRange(local, inv, this.blasNode(d, sub, lid));
            const r = this.aabbRange(local, inv, this.blasNode(d, sub, rid));
            const lh = vx <= l[1] && l[0] <= vy, rh = vx <= r[1] && r[0] <= vy;
            if (lh && rh) {
              if (l[0] < r[0]) { stack[++sp] = rid; stack[++sp] = lid; } else { stack[++sp] = lid; stack[++sp] = rid; }
            } else if (lh) stack[++sp] = lid;
            else if (rh) stack[++sp] = rid;
            continue;
          }
          const first = A[node + 6], last = first + (A[node + 7] & 0xffff);
          for (let prim = first; prim < last; ++prim) {
            const ids = this.triIds(d, prim);
            const t = this.rayTri(local, this.vpos(d, ids[0]), this.vpos(d, ids[1]), this.vpos(d, ids[2]));
            if (vy < t) continue;
            vy = t; valid = true; binst = inst; bsub = sub; bprim = prim;
          }
        }
      }
    }
    const hit = { valid, t: 0, s: { valid: valid ? 1 : 0, inst: binst, mat: bsub, prim: bprim, bu: 0, bv: 0 } };
    if (valid) {
      hit.t = vy;
      const d = this.desc(this.instMesh(binst)), mo = STRIDE_INSTANCE * binst;
      const ids = this.triIds(d, bprim);
      const A0 = xformPoint(F, mo, this.vpos(d, ids[0])), B = xformPoint(F, mo, this.vpos(d, ids[1]));
      const C = xformPoint(F, mo, this.vpos(d, ids[2]));
      const P = vadd(ray.o, vscale(ray.d, vy));
      // GetBaryCentricWeights, PT_1:549-575
      const v0 = vsub(B, A0), v1 = vsub(C, A0), v2 = vsub(P, A0);
      const d00 = vdot(v0, v0), d01 = vdot(v0, v1), d11 = vdot(v1, v1), d20 = vdot(v2, v0), d21 = vdot(v2, v1);
      const denom = f(f(d00 * d11) - f(d01 * d01));
      if (Math.abs(denom) < this.eps.bary) { hit.s.bu = 1; hit.s.bv = 0; } else {
        const inv = f(1 / denom);
        const u = f(f(f(d11 * d20) - f(d01 * d21)) * inv), v = f(f(f(d00 * d21) - f(d01 * d20)) * inv);
        hit.s.bu = f(f(1 - u) - v);
        hit.s.bv = u;
      }
    }
    return hit;
  }

  // ------------------------------------------------------------ lights
  light(id) {
    const o = this.U[U_OFF_LIGHT] + STRIDE_LIGHT * id, F = this.Sf;
    return { pos: V3(F[o], F[o + 1], F[o + 2]), dir: V3(F[o + 3], F[o + 4], F[o + 5]), color: V3(F[o + 6], F[o + 7], F[o + 8]),
      U: V3(F[o + 9], F[o + 10], F[o + 11]), V: V3(F[o + 12], F[o + 13], F[o + 14]), type: this.S[o + 15], intensity: F[o + 16], area: F[o + 17] };
  }
  lightCdf(i) { return this.Sf[this.U[U_OFF_CDF] + i]; }
  dirToLight(X, XL) { // DirectionToLight, PT_1:746-772
    if (XL.type === LIGHT_DIRECTION || XL.type === LIGHT_ENV) return vneg(XL.dir);
    if (XL.type === LIGHT_POINT || XL.type === LIGHT_RECT) return vnormalize(vsub(XL.pos, X.pos));
    return V3(0, 0, 0);
  }
  pdfLight(X, V, XL) { // PDF_LIGHT, PT_1:1220-1245 (PT_4:1249 drops the EPS guard)
    if (XL.type === LIGHT_ENV) return pdfBsdf(X, V, this.dirToLight(X, XL));
    const ls = this.light(XL.id);
    const before = XL.id === 0 ? 0 : this.lightCdf(XL.id - 1);
    const choose = f(this.lightCdf(XL.id) - before);
    let pdfPoint = 1;
    if (XL.type === LIGHT_RECT) {
      const r = vsub(XL.pos, X.pos), L = vnormalize(r);
      const denom = f(ls.area * Math.abs(vdot(ls.dir, L)));
      pdfPoint = f(vdot(r, r) / (this.eps.final ? denom : fmax(denom, EPS_F)));
    }
    return f(choose * pdfPoint);
  }
  sampleNee(st, X, V) { // SampleNEE, PT_1:970-1025
    const P = random(st);
    let L = 0, R = this.U[U_LIGHT_COUNT] - 1, M = (L + R) >>> 1;
    while (L < R) {
      if (P < this.lightCdf(M)) R = M; else L = M + 1;
      M = (L + R) >>> 1;
    }
    const ls = this.light(M);
    const s = { id: M, type: ls.type, Le: vscale(ls.color, ls.intensity), pos: V3(0, 0, 0), dir: V3(0, 0, 0), pdf: 0 };
    if (ls.type === LIGHT_DIRECTION) { s.pos = vsub(X.pos, vscale(ls.dir, INF_F)); s.dir = ls.dir; }
    else if (ls.type === LIGHT_POINT) { s.pos = ls.pos; s.dir = vnormalize(vsub(X.pos, ls.pos)); }
    else if (ls.type === LIGHT_RECT) {
      const ru = f(f(random(st) * 2) - 1), rv = f(f(random(st) * 2) - 1);
      s.pos = vadd(ls.pos, vadd(vscale(ls.U, ru), vscale(ls.V, rv)));
      s.dir = vnormalize(vsub(X.pos, s.pos));
    }
    s.pdf = this.pdfLight(X, V, s);
    return s;
  }
  lEmit(XL, X) { // L_emit, PT_1:1253-1260 (PT_4:1265 unguarded)
    const r = vsub(XL.pos, X.pos), rr = vdot(r, r);
    const att = XL.type === LIGHT_POINT ? f(1 / (this.eps.final ? rr : fmax(rr, EPS_F))) : 1;
    return vscale(XL.Le, att);
  }
  visibility(start, end) { // Visibility + GetMaterialFromHit, PT_1:316-322,774-802
    let T = 1;
    const dist = vlength(vsub(end, start));
    const ray = { o: start, d: vdivs(vsub(end, start), dist) };
    let remain = dist;
    for (let it = 0; it < 5; ++it) {
      const h = this.trace(ray);
      if (!h.valid || h.t > remain) return T;
      const m = this.material(this.desc(this.instMesh(h.s.inst)), h.s.mat);
      if (m.trans === 0) return 0;
      T = f(T * m.trans);
      remain = f(remain - h.t);
      ray.o = this.surface(h.s).pos;
    }
    return 0;
  }

  // ------------------------------------------------------------ camera
  x0(x, y) { // Get_X0, PT_1:732-738
    const u = f(f(x + 0.5) / f(this.W)), v = f(f(y + 0.5) / f(this.H));
    return xformPoint(this.uf(), U_VPINV, V3(f(f(2 * u) - 1), f(f(2 * v) - 1), 0));
  }
  uf() { if (!this._uf) this._uf = new Float32Array(this.U.buffer, this.U.byteOffset, this.U.length); return this._uf; }
  cameraRay(x, y) { // GenerateRayFromThreadID, PT_01:496-507
    const u = f(f(x + 0.5) / f(this.W)), v = f(f(y + 0.5) / f(this.H));
    const o = V3(f(f(2 * u) - 1), f(f(2 * v) - 1), 0);
    const start = xformPoint(this.uf(), U_VPINV, o), end = xformPoint(this.uf(), U_VPINV, vadd(o, V3(0, 0, 1)));
    return { o: start, d: vnormalize(vsub(end, start)) };
  }
  initSeed(x, y) { return pcg((Math.imul(x, 1973) + Math.imul(y, 9277) + Math.imul(this.U[U_FRAME], 26699)) >>> 0); }

  // ------------------------------------------------------------ PT_01
  gbufferPixel(x, y, out, o) {
    this.eps = EPS_GBUFFER;
    const h = this.trace(this.cameraRay(x, y));
    out[o] = (((h.valid ? 1 : 0) << 31) | (h.s.inst << 16) | h.s.mat) >>> 0;
    out[o + 1] = h.s.prim;
    f32v[0] = h.s.bu; out[o + 2] = u32v[0];
    f32v[0] = h.s.bv; out[o + 3] = u32v[0];
  }

  // ------------------------------------------------------------ PT_1
  initPixel(gb, x, y, res, ro) {
    this.eps = EPS_INIT;
    const go = 4 * (y * this.W + x);
    const x1 = decode(gb, go);
    res.fill(0, ro, ro + 32);
    if (!x1.valid) return; // PT_4 returns before LoadReservoir (:1404-1408)
    const st = { s: this.initSeed(x, y) };
    let fT = V3(1, 1, 0 + 1), p = 1;
    const ps = { pos: [], rough: [0, 0, 0, 0], lobe: [0, 0, 0, 0], nee: [0, 0, 0, 0], bsdf: [0, 0, 0, 0], cs: [] };
    const X = [];
    ps.cs[1] = x1;
    X[0] = { pos: this.x0(x, y) };
    X[1] = this.surface(x1);
    ps.pos[0] = X[0].pos; ps.pos[1] = X[1].pos; ps.rough[1] = X[1].mat.rough;
    let C = 0, wSum = 0, pSel = 0, selI = -1, selEnv = false, selXL = null;
    for (let i = 1; i < 4; ++i) {
      const S = X[i];
      const V = vnormalize(vsub(X[i - 1].pos, S.pos));
      ps.nee[i] = st.s;
      const XL = this.sampleNee(st, S, V);
      let L = this.dirToLight(S, XL);
      let contrib = vmul(fT, this.lEmit(XL, S));
      contrib = vmul(contrib, bsdf(S, V, L));
      contrib = vscale(contrib, Math.abs(vdot(S.nrm, L)));
      contrib = vscale(contrib, this.visibility(S.pos, XL.pos));
      const pHat = luminance(contrib);
      const ris = f(pHat / f(p * XL.pdf));
      C += 1; // UpdateReservoir, PT_1:1298-1320
      wSum = f(wSum + ris);
      if (random(st) < f(ris / wSum)) { selI = i; selEnv = false; selXL = XL; pSel = pHat; }
      if (i === 3) break;
      ps.bsdf[i] = st.s;
      const lb = { lobe: 0 };
      L = sampleBsdf(st, S, V, lb);
      ps.lobe[i] = lb.lobe;
      const b = vscale(bsdf(S, V, L), Math.abs(vdot(S.nrm, L)));
      fT = vmul(fT, b);
      p = f(p * pdfBsdf(S, V, L));
      const pSurv = f(luminance(fT) / p);
      if (random(st) < pSurv) p = f(p * pSurv); else break;
      const h = this.trace({ o: S.pos, d: L });
      if (!h.valid) { // env candidate, PT_1:1447-1461
        const env = { pos: vadd(S.pos, vscale(L, INF_F)), type: LIGHT_ENV, dir: vneg(L), id: -1, Le: V3(ENV_C, ENV_C, ENV_C), pdf: pdfBsdf(S, V, L) };
        const ph = luminance(vscale(fT, ENV_C));
        const risE = f(ph / p);
        C += 1;
        wSum = f(wSum + risE);
        if (random(st) < f(risE / wSum)) { selI = i; selEnv = true; selXL = env; pSel = ph; }
        break;
      }
      ps.cs[i + 1] = h.s;
      X[i + 1] = this.surface(h.s);
      ps.pos[i + 1] = X[i + 1].pos; ps.rough[i + 1] = X[i + 1].mat.rough;
    }
    if (selI >= 0) this.compress(ps, selI, selEnv, selXL, res, ro);
    f32v[0] = f(wSum / pSel); res[ro + 28] = u32v[0];
    res[ro + 29] = C;
  }
  compress(ps, i, isEnv, XL, out, o) { // CompressPath + SafeReconnectionIndex, PT_1:1262-1353
    const lobe = [0, 0, 0, 0, 0, 0, 0, 0], seed = [0, 0, 0, 0, 0, 0, 0, 0];
    for (let k = 1; k < i; ++k) { lobe[k] = ps.lobe[k]; seed[k + 1] = ps.bsdf[k]; }
    if (isEnv) { lobe[i] = ps.lobe[i]; seed[i + 1] = ps.bsdf[i]; } else seed[i + 1] = ps.nee[i];
    const length = i + 1;
    let k = 0;
    for (let kk = 2; kk < length; ++kk) {
      const ra = lobe[kk - 1] === LOBE_LAMBERT ? 1 : ps.rough[kk - 1];
      const rb = lobe[kk] === LOBE_LAMBERT ? 1 : ps.rough[kk];
      const rough = fmin(ra, rb) >= RECONNECTION_ROUGHNESS;
      const far = vlength(vsub(ps.pos[kk - 1], ps.pos[kk])) >= RECONNECTION_DISTANCE;
      if (far && rough) { k = kk; break; }
    }
    if (k === 0) {
      const rough = ps.rough[length - 1] >= RECONNECTION_ROUGHNESS;
      const dirl = XL.type === LIGHT_DIRECTION || XL.type === LIGHT_ENV;
      const far = dirl || vlength(vsub(ps.pos[length - 1], XL.pos)) >= RECONNECTION_DISTANCE;
      if (far && rough) k = length;
    }
    out[o] = seed[2] >>> 0; out[o + 1] = seed[3] >>> 0; out[o + 2] = seed[4] >>> 0; out[o + 3] = seed[5] >>> 0;
    putF(out, o + 4, [XL.dir.x, XL.dir.y, XL.dir.z]); out[o + 7] = XL.type;
    putF(out, o + 8, [XL.pos.x, XL.pos.y, XL.pos.z]); out[o + 11] = XL.id >>> 0;
    putF(out, o + 12, [XL.Le.x, XL.Le.y, XL.Le.z, XL.pdf]);
    out[o + 20] = k; out[o + 23] = length;
    if (k !== 0) {
      const isLight = k === length;
      out[o + 22] = isLight ? LOBE_LIGHT : lobe[k];
      out[o + 21] = lobe[k - 1];
      if (!isLight) {
        const c = ps.cs[k];
        out[o + 16] = ((c.valid << 31) | (c.inst << 16) | c.mat) >>> 0; out[o + 17] = c.prim;
        putF(out, o + 18, [c.bu, c.bv]);
      }
    }
  }

  // ------------------------------------------------------------ PT_4
  finalPixel(gb, res, x, y, accum) {
    this.eps = EPS_FINAL;
    const p = y * this.W + x, go = 4 * p, ro = 32 * p, ao = 4 * p;
    const x1 = decode(gb, go);
    if (!x1.valid) { accum[ao] = ENV_C; accum[ao + 1] = ENV_C; accum[ao + 2] = ENV_C; accum[ao + 3] = 1; return; }
    const C = res[ro + 29], length = res[ro + 23];
    if (C === 0 || length < 2) { this.writeColor(accum, ao, V3(0, 0, 0)); return; }
    const F = new Float32Array(res.buffer, res.byteOffset + 4 * ro, 32);
    const XL = { dir: V3(F[4], F[5], F[6]), type: res[ro + 7], pos: V3(F[8], F[9], F[10]), id: res[ro + 11] | 0, Le: V3(F[12], F[13], F[14]), pdf: F[15] };
    const S = [];
    S[0] = { pos: this.x0(x, y) };
    S[1] = this.surface(x1);
    for (let i = 1; i + 1 < length; ++i) { // RegeneratePath, PT_4:1357-1384
      const V = vnormalize(vsub(S[i - 1].pos, S[i].pos));
      const st = { s: res[ro + i - 1] };
      const dir = sampleBsdf(st, S[i], V, { lobe: 0 });
      const h = this.trace({ o: S[i].pos, d: dir });
      S[i + 1] = this.surface(h.s); // a miss decodes the zero CompactSurface, as the WGSL does
    }
    let fT = V3(1, 1, 1); // PathContribution, PT_4:1306-1336
    for (let i = 1; i + 1 < length; ++i) {
      const V = vnormalize(vsub(S[i - 1].pos, S[i].pos)), L = vnormalize(vsub(S[i + 1].pos, S[i].pos));
      fT = vmul(fT, vscale(bsdf(S[i], L, V), Math.abs(vdot(S[i].nrm, L))));
    }
    const P = S[length - 2], Xc = S[length - 1];
    const V = vnormalize(vsub(P.pos, Xc.pos)), L = this.dirToLight(Xc, XL);
    fT = vmul(fT, vscale(bsdf(Xc, L, V), Math.abs(vdot(Xc.nrm, L))));
    fT = vmul(fT, vscale(this.lEmit(XL, Xc), this.visibility(Xc.pos, XL.pos)));
    this.writeColor(accum, ao, vscale(fT, F[28]));
  }
  writeColor(accum, o, c) { // WriteColor, PT_4:599-606
    const t = f(1 / f(this.U[U_FRAME] + 1));
    accum[o] = mixf(accum[o], c.x, t); accum[o + 1] = mixf(accum[o + 1], c.y, t); accum[o + 2] = mixf(accum[o + 2], c.z, t);
    accum[o + 3] = 1;
  }

  /** One ReSTIR frame over rows [y0, y1) (rows also striped: y = y0 + k * step). */
  frameRows(rows, gb, res, accum) {
    const W = this.W;
    for (const y of rows) for (let x = 0; x < W; ++x) this.gbufferPixel(x, y, gb, 4 * (y * W + x));
    for (const y of rows) for (let x = 0; x < W; ++x) this.initPixel(gb, x, y, res, 32 * (y * W + x));
    for (const y of rows) for (let x = 0; x < W; ++x) this.finalPixel(gb, res, x, y, accum);
  }
}

// ---------------------------------------------------------------- BSDF, PT_1:834-929
function ggxD(NdotH, R) {
  const a = f(R * R), a2 = f(a * a);
  const X = f(f(f(NdotH * NdotH) * f(a2 - 1)) + 1);
  const denom = f(f(PI_F * X) * X);
  return f(a2 / fmax(denom, EPS_F));
}
function geomShadow(NdotV, NdotL, R) {
  const r = f(R + 1), K = f(f(r * r) / 8);
  return f(1 / f(f(f(NdotV * f(1 - K)) + K) * f(f(NdotL * f(1 - K)) + K)));
}
function fresnel(d, F0) {
  const p = pow5(f(1 - saturate(d)));
  return V3(f(F0.x + f(f(1 - F0.x) * p)), f(F0.y + f(f(1 - F0.y) * p)), f(F0.z + f(f(1 - F0.z) * p)));
}
const F004 = V3(f(0.04), f(0.04), f(0.04));
function brdf(X, V, L) {
  const N = X.nrm, H = vnormalize(vadd(L, V));
  const NdotV = fmax(vdot(N, V), 0), NdotL = fmax(vdot(N, L), 0), NdotH = fmax(vdot(N, H), 0), VdotH = fmax(vdot(V, H), 0);
  const base = X.mat.albedo, metal = X.mat.metal, R = X.mat.rough;
  const F0 = vmix(F004, base, metal);
  const D = ggxD(NdotH, R), G0 = geomShadow(NdotV, NdotL, R), F = fresnel(VdotH, F0);
  const kD = vscale(V3(f(1 - F.x), f(1 - F.y), f(1 - F.z)), f(1 - metal));
  const diffuse = vmul(vdivs(kD, PI_F), base);
  const spec = vscale(vscale(vscale(F, D), G0), f(0.25));
  return vadd(diffuse, spec);
}
function btdf(X, V, L) {
  const albedo = X.mat.albedo, R = X.mat.rough;
  const same = vdot(V, X.nrm) > 0;
  const nIn = same ? X.mat.ior : 1, nOut = same ? 1 : X.mat.ior;
  const hv = vadd(vscale(L, nIn), vscale(V, nOut));
  const Hn = vlength(hv);
  const N = same ? X.nrm : vneg(X.nrm), H = vnormalize(hv);
  const NdotL = Math.abs(vdot(N, L)), NdotV = Math.abs(vdot(N, V)), NdotH = Math.abs(vdot(N, H));
  const LdotH = Math.abs(vdot(L, H)), VdotH = Math.abs(vdot(V, H));
  const G0 = geomShadow(NdotL, NdotV, R), D = ggxD(NdotH, R);
  const nr = f(f(nOut - nIn) / f(nOut + nIn)), n2 = f(nr * nr);
  const F = fresnel(LdotH, V3(n2, n2, n2));
  let num = vscale(V3(f(1 - F.x), f(1 - F.y), f(1 - F.z)), f(nOut * nOut));
  num = vscale(num, LdotH); num = vscale(num, VdotH); num = vscale(num, G0); num = vscale(num, D);
  num = vmul(num, albedo);
  void NdotL;
  return vdivs(num, fmax(f(Hn * Hn), EPS_F));
}
function bsdf(X, V, L) {
  const T = X.mat.trans, N = X.nrm;
  if (f(vdot(L, N) * vdot(V, N)) > 0) return vscale(brdf(X, V, L), f(1 - T));
  return vscale(btdf(X, V, L), T);
}
// ---------------------------------------------------------------- sampling, PT_1:577-589,937-1106
function tbn(N) {
  const same = Math.abs(vdot(N, V3(0, 1, 0))) > f(0.9999);
  const cv = same ? V3(1, 0, 0) : V3(0, 1, 0);
  const T = vnormalize(vcross(cv, N));
  return { T, B: vcross(N, T), N };
}
const m3mul = (m, v) => vadd(vadd(vscale(m.T, v.x), vscale(m.B, v.y)), vscale(m.N, v.z));
const reflect = (I, N) => vsub(I, vscale(N, f(2 * vdot(N, I))));
function refract(I, N, eta) {
  const d = vdot(N, I);
  const k = f(1 - f(f(eta * eta) * f(1 - f(d * d))));
  if (k < 0) return V3(0, 0, 0);
  return vsub(vscale(I, eta), vscale(N, f(f(eta * d) + f(Math.sqrt(k)))));
}
const TWO_PI = f(2 * PI_F);
function sampleCosine(st) {
  const r1 = random(st), r2 = random(st);
  const R = f(Math.sqrt(r1));
  const [sp, cp] = sincos(f(TWO_PI * r2));
  return V3(f(R * cp), f(R * sp), f(Math.sqrt(f(1 - r1))));
}
function sampleGgx(st, R) {
  const r1 = random(st), r2 = random(st);
  const a = f(R * R);
  const phi = f(TWO_PI * r1);
  const ct = f(Math.sqrt(f(f(1 - r2) / f(1 + f(f(f(a * a) - 1) * r2)))));
  const stt = f(Math.sqrt(f(1 - f(ct * ct))));
  const [sp, cp] = sincos(phi);
  return vnormalize(V3(f(stt * cp), f(stt * sp), ct));
}
function sampleBrdf(st, X, V, lb) {
  const metal = X.mat.metal;
  const F0 = vmix(F004, X.mat.albedo, metal);
  const pSpec = mixf(luminance(F0), 1, metal);
  const m = tbn(X.nrm);
  const spec = random(st) < pSpec;
  let L;
  if (spec) L = reflect(vneg(V), m3mul(m, sampleGgx(st, X.mat.rough)));
  else L = m3mul(m, sampleCosine(st));
  lb.lobe = spec ? LOBE_GGX : LOBE_LAMBERT;
  return L;
}
function sampleBtdf(st, X, V, lb) {
  const same = vdot(V, X.nrm) > 0;
  const nIn = same ? 1 : X.mat.ior, nOut = same ? X.mat.ior : 1;
  const N = same ? X.nrm : vneg(X.nrm);
  const ratio = f(nIn / nOut), r = f(f(1 - ratio) / f(1 + ratio)), R2 = f(ratio * ratio);
  const cosT = Math.abs(vdot(V, N));
  const rr = f(r * r);
  let pRefl = fresnel(cosT, V3(rr, rr, rr)).x;
  if (f(cosT * cosT) < f(f(R2 - 1) / R2)) pRefl = 1;
  const refl = random(st) < pRefl;
  const m = tbn(N);
  const H = m3mul(m, sampleGgx(st, X.mat.rough));
  const Lr = refract(vneg(V), H, ratio), Ll = reflect(vneg(V), H);
  lb.lobe = LOBE_GGX;
  return vnormalize(refl ? Ll : Lr);
}
function sampleBsdf(st, X, V, lb) {
  const transparent = random(st) < X.mat.trans;
  return transparent ? sampleBtdf(st, X, V, lb) : sampleBrdf(st, X, V, lb);
}
// ---------------------------------------------------------------- pdfs, PT_1:1114-1245
function pdfBrdf(X, V, L) {
  const metal = X.mat.metal, R = X.mat.rough;
  const F0 = vmix(F004, X.mat.albedo, metal);
  const pSpec = mixf(luminance(F0), 1, metal);
  const N = X.nrm, H = vnormalize(vadd(L, V));
  const LdotN = fmax(vdot(L, N), 0), NdotH = fmax(vdot(N, H), 0), VdotH = fmax(vdot(V, H), 0);
  const pdfS = f(ggxD(NdotH, R) / fmax(f(4 * VdotH), EPS_F));
  const pdfD = f(LdotN / PI_F);
  return mixf(pdfD, pdfS, pSpec);
}
function pdfBtdf(X, V, L) {
  const R = X.mat.rough;
  const same = vdot(V, X.nrm) > 0;
  const nIn = same ? 1 : X.mat.ior, nOut = same ? X.mat.ior : 1;
  const ratio = f(nIn / nOut);
  const N = same ? X.nrm : vneg(X.nrm);
  const r0 = f(f(1 - ratio) / f(1 + ratio)), R0 = f(r0 * r0);
  const cosT = Math.abs(vdot(V, N));
  let pRefl = fresnel(cosT, V3(R0, R0, R0)).x;
  const sin2 = f(1 - f(cosT * cosT)), R2 = f(ratio * ratio);
  if (f(sin2 * R2) > 1) pRefl = 1;
  const pTrans = f(1 - pRefl);
  let pdfR = 0;
  if (pRefl > 0) {
    const Hr = vnormalize(vadd(V, L));
    const NdotHr = fmax(0, vdot(N, Hr)), VdotHr = fmax(0, vdot(V, Hr));
    if (VdotHr > 0) pdfR = f(ggxD(NdotHr, R) / f(4 * VdotHr));
  }
  let pdfT = 0;
  if (pTrans > 0) {
    const Ht = vnormalize(vadd(vscale(V, nOut), vscale(L, nIn)));
    const NdotHt = fmax(0, vdot(N, Ht)), VdotHt = fmax(0, vdot(V, Ht)), LdotHt = fmax(0, vdot(L, Ht));
    const denom = f(f(nIn * LdotHt) + f(nOut * VdotHt));
    if (denom > 0) {
      const J = f(f(f(nOut * nOut) * VdotHt) / f(denom * denom));
      pdfT = f(ggxD(NdotHt, R) * Math.abs(J));
    }
  }
  return f(f(pRefl * pdfR) + f(pTrans * pdfT));
}
function pdfBsdf(X, V, L) {
  const N = X.nrm;
  if (f(vdot(L, N) * vdot(V, N)) > 0) return pdfBrdf(X, V, L);
  return pdfBtdf(X, V, L);
}

// ---------------------------------------------------------------- buffers
const f32v = new Float32Array(1), u32v = new Uint32Array(f32v.buffer);
function putF(out, o, vals) { for (let i = 0; i < vals.length; ++i) { f32v[0] = vals[i]; out[o + i] = u32v[0]; } }
function decode(gb, o) { // GetCompactSurface, PT_1:424-436
  const w = gb[o];
  u32v[0] = gb[o + 2]; const bu = f32v[0];
  u32v[0] = gb[o + 3]; const bv = f32v[0];
  return { valid: (w & 0x80000000) !== 0 ? 1 : 0, inst: (w & 0x7fff0000) >>> 16, mat: w & 0xffff, prim: gb[o + 1], bu, bv };
}

module.exports = { CpuTracer, pcg, sincos, pow5 };
