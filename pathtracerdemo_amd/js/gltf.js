'use strict';
/**
 * Mesh.Load for the Node host (GC/Structs.ts:108-141): read a binary glTF, visit every mesh
 * of its default scene depth-first (traverseGLTF, :118-124; one THREE.Mesh per primitive),
 * bake each node's world matrix into positions and normals (geometry.applyMatrix4, :132),
 * merge the primitives with one group per primitive (mergeGeometries(geoms, true), :139) and
 * read the MeshStandardMaterial fields Material's constructor uses (GLTFLoader defaults).
 *
 * three@0.180.0 is not installed here: the matrix arithmetic is restated in three.js's own
 * operation order (Matrix4.compose / multiplyMatrices, Matrix3.getNormalMatrix, Vector3
 * .applyMatrix4 / applyMatrix3 / normalize, f64 math stored to f32 attributes), exactly as the
 * Python scene compiler does (pathtracerdemo_amd/scene/gltf.py), so both hosts produce the same
 * bits (tests/test_node_host.py).  The SAH BLAS build is ./bvh.js.
 */
const fs = require('fs');

const COMPONENT = { 5120: Int8Array, 5121: Uint8Array, 5122: Int16Array, 5123: Uint16Array, 5125: Uint32Array,
  5126: Float32Array };
const GETTER = { 5120: 'getInt8', 5121: 'getUint8', 5122: 'getInt16', 5123: 'getUint16', 5125: 'getUint32',
  5126: 'getFloat32' };
const NCOMP = { SCALAR: 1, VEC2: 2, VEC3: 3, VEC4: 4, MAT4: 16 };

/** The GLB container: its JSON chunk and binary chunk. */
function readGlb(file) {
  const data = fs.readFileSync(file);
  const dv = new DataView(data.buffer, data.byteOffset, data.byteLength);
  if (dv.getUint32(0, true) !== 0x46546C67 || dv.getUint32(4, true) !== 2) throw new Error(`${file}: not a glTF 2.0 binary`);
  const length = dv.getUint32(8, true);
  let json = null;
  let bin = Buffer.alloc(0);
  for (let off = 12; off < length;) {
    const clen = dv.getUint32(off, true), ctype = dv.getUint32(off + 4, true);
    const chunk = data.subarray(off + 8, off + 8 + clen);
    if (ctype === 0x4E4F534A) json = JSON.parse(chunk.toString('utf8'));
    else if (ctype === 0x004E4942) bin = chunk;
    off += 8 + clen;
  }
  if (!json) throw new Error(`${file}: missing JSON chunk`);
  return { json, bin };
}

/** Accessor idx as a flat array of count * ncomp elements (a copy; byteStride honoured). */
function accessor(g, idx) {
  const acc = g.json.accessors[idx];
  const T = COMPONENT[acc.componentType], ncomp = NCOMP[acc.type], count = acc.count;
  if (!T || !ncomp) throw new Error(`accessor ${idx}: unsupported type`);
  if (acc.normalized) throw new Error('normalized accessors are not supported');
  const out = new T(count * ncomp);
  if (acc.bufferView === undefined) return { data: out, count, ncomp };
  const bv = g.json.bufferViews[acc.bufferView];
  if ((bv.buffer || 0) !== 0) throw new Error('external buffers are not supported');
  const start = (bv.byteOffset || 0) + (acc.byteOffset || 0);
  const esize = T.BYTES_PER_ELEMENT, stride = bv.byteStride || esize * ncomp;
  const dv = new DataView(g.bin.buffer, g.bin.byteOffset, g.bin.byteLength);
  const get = GETTER[acc.componentType];
  for (let i = 0; i < count; i++)
    for (let c = 0; c < ncomp; c++) out[i * ncomp + c] = dv[get](start + i * stride + c * esize, true);
  return { data: out, count, ncomp };
}

/** Matrix4.compose(position, quaternion, scale), column-major. */
function compose(t, q, s) {
  const [x, y, z, w] = q, [sx, sy, sz] = s;
  const x2 = x + x, y2 = y + y, z2 = z + z;
  const xx = x * x2, xy = x * y2, xz = x * z2;
  const yy = y * y2, yz = y * z2, zz = z * z2;
  const wx = w * x2, wy = w * y2, wz = w * z2;
  return [(1 - (yy + zz)) * sx, (xy + wz) * sx, (xz - wy) * sx, 0,
    (xy - wz) * sy, (1 - (xx + zz)) * sy, (yz + wx) * sy, 0,
    (xz + wy) * sz, (yz - wx) * sz, (1 - (xx + yy)) * sz, 0,
    t[0], t[1], t[2], 1];
}

/** The sign-relevant 4x4 determinant (cofactor expansion along the first row). */
function determinant(m) {
  const a = (r, c) => m[4 * c + r];
  const det3 = (r0, r1, r2, c0, c1, c2) => a(r0, c0) * (a(r1, c1) * a(r2, c2) - a(r1, c2) * a(r2, c1))
    - a(r0, c1) * (a(r1, c0) * a(r2, c2) - a(r1, c2) * a(r2, c0)) + a(r0, c2) * (a(r1, c0) * a(r2, c1) - a(r1, c1) * a(r2, c0));
  return a(0, 0) * det3(1, 2, 3, 1, 2, 3) - a(0, 1) * det3(1, 2, 3, 0, 2, 3)
    + a(0, 2) * det3(1, 2, 3, 0, 1, 3) - a(0, 3) * det3(1, 2, 3, 0, 1, 2);
}

/** Matrix4.decompose(position, quaternion, scale) with Quaternion.setFromRotationMatrix (f64). */
function decompose(m) {
  let sx = Math.sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
  const sy = Math.sqrt(m[4] * m[4] + m[5] * m[5] + m[6] * m[6]);
  const sz = Math.sqrt(m[8] * m[8] + m[9] * m[9] + m[10] * m[10]);
  if (determinant(m) < 0) sx = -sx;
  const ix = 1 / sx, iy = 1 / sy, iz = 1 / sz;
  const m11 = m[0] * ix, m21 = m[1] * ix, m31 = m[2] * ix;
  const m12 = m[4] * iy, m22 = m[5] * iy, m32 = m[6] * iy;
  const m13 = m[8] * iz, m23 = m[9] * iz, m33 = m[10] * iz;
  const trace = m11 + m22 + m33;
  let q;
  if (trace > 0) {
    const s = 0.5 / Math.sqrt(trace + 1.0);
    q = [(m32 - m23) * s, (m13 - m31) * s, (m21 - m12) * s, 0.25 / s];
  } else if (m11 > m22 && m11 > m33) {
    const s = 2.0 * Math.sqrt(1.0 + m11 - m22 - m33);
    q = [0.25 * s, (m12 + m21) / s, (m13 + m31) / s, (m32 - m23) / s];
  } else if (m22 > m33) {
    const s = 2.0 * Math.sqrt(1.0 + m22 - m11 - m33);
    q = [(m12 + m21) / s, 0.25 * s, (m23 + m32) / s, (m13 - m31) / s];
  } else {
    const s = 2.0 * Math.sqrt(1.0 + m33 - m11 - m22);
    q = [(m13 + m31) / s, (m23 + m32) / s, 0.25 * s, (m21 - m12) / s];
  }
  return { t: [m[12], m[13], m[14]], q, s: [sx, sy, sz] };
}

/** A node's local matrix as three.js ends up composing it.  A glTF `matrix` goes through
 * GLTFLoader's node.applyMatrix4: premultiplied onto the identity, decomposed, and recomposed by
 * updateMatrix -- the raw matrix itself is never used (as scene/gltf.py; restated from three's
 * published source, parity-unpinned against the library, which is not installed here). */
function localMatrix(node) {
  if (node.matrix) {
    const d = decompose(multiply(node.matrix.slice(), compose([0, 0, 0], [0, 0, 0, 1], [1, 1, 1])));
    return compose(d.t, d.q, d.s);
  }
  return compose(node.translation || [0, 0, 0], node.rotation || [0, 0, 0, 1], node.scale || [1, 1, 1]);
}

/** Matrix4.multiplyMatrices(a, b), column-major. */
function multiply(a, b) {
  const out = new Array(16);
  for (let r = 0; r < 4; r++)
    for (let c = 0; c < 4; c++)
      out[4 * c + r] = a[r] * b[4 * c] + a[4 + r] * b[4 * c + 1] + a[8 + r] * b[4 * c + 2] + a[12 + r] * b[4 * c + 3];
  return out;
}

/** Matrix3.getNormalMatrix(m): the upper 3x3 inverted by cofactors, transposed (zeros if singular). */
function normalMatrix(m) {
  const n11 = m[0], n21 = m[1], n31 = m[2], n12 = m[4], n22 = m[5], n32 = m[6], n13 = m[8], n23 = m[9], n33 = m[10];
  const t11 = n33 * n22 - n32 * n23, t12 = n32 * n13 - n33 * n12, t13 = n23 * n12 - n22 * n13;
  const det = n11 * t11 + n21 * t12 + n31 * t13;
  if (det === 0) return new Array(9).fill(0);
  const d = 1 / det;
  const inv = [t11 * d, (n31 * n23 - n33 * n21) * d, (n32 * n21 - n31 * n22) * d,
    t12 * d, (n33 * n11 - n31 * n13) * d, (n31 * n12 - n32 * n11) * d,
    t13 * d, (n21 * n13 - n23 * n11) * d, (n22 * n11 - n21 * n12) * d];
  return [inv[0], inv[3], inv[6], inv[1], inv[4], inv[7], inv[2], inv[5], inv[8]];
}

/** MeshStandardMaterial fields as GLTFLoader sets them (the subset Material reads, Structs.ts:311-320). */
function material(g, idx) {
  if (idx === undefined) {
    return { color: { r: 1, g: 1, b: 1 }, emissive: { r: 0, g: 0, b: 0 }, emissiveIntensity: 1, metalness: 1,
      roughness: 1, transparent: false };
  }
  const m = g.json.materials[idx];
  const pbr = m.pbrMetallicRoughness || {};
  const bc = pbr.baseColorFactor || [1, 1, 1, 1], em = m.emissiveFactor || [0, 0, 0];
  const ext = m.extensions || {};
  const strength = (ext.KHR_materials_emissive_strength || {}).emissiveStrength;
  return {
    color: { r: bc[0], g: bc[1], b: bc[2] }, emissive: { r: em[0], g: em[1], b: em[2] },
    emissiveIntensity: strength === undefined ? 1 : strength,
    metalness: pbr.metallicFactor === undefined ? 1 : pbr.metallicFactor,
    roughness: pbr.roughnessFactor === undefined ? 1 : pbr.roughnessFactor,
    transparent: (m.alphaMode || 'OPAQUE') === 'BLEND',
  };
}

/** geometry.applyMatrix4(matrixWorld): positions through Vector3.applyMatrix4, normals through the
 * normal matrix then normalize() (divideScalar(length() || 1) = multiplyScalar(1 / len)), f64 math, f32 storage. */
function bake(g, prim, e) {
  const attrs = prim.attributes;
  const P = accessor(g, attrs.POSITION), nv = P.count;
  if (attrs.NORMAL === undefined) throw new Error('primitives without normals are not supported');
  const N = accessor(g, attrs.NORMAL);
  const uv = attrs.TEXCOORD_0 !== undefined ? new Float32Array(accessor(g, attrs.TEXCOORD_0).data) : null;
  const index = prim.indices !== undefined ? Uint32Array.from(accessor(g, prim.indices).data)
    : Uint32Array.from({ length: nv }, (_, i) => i);
  const positions = new Float32Array(3 * nv), normals = new Float32Array(3 * nv);
  const n = normalMatrix(e);
  for (let v = 0; v < nv; v++) {
    const x = P.data[3 * v], y = P.data[3 * v + 1], z = P.data[3 * v + 2];
    const w = 1 / (e[3] * x + e[7] * y + e[11] * z + e[15]);
    positions[3 * v] = (e[0] * x + e[4] * y + e[8] * z + e[12]) * w;
    positions[3 * v + 1] = (e[1] * x + e[5] * y + e[9] * z + e[13]) * w;
    positions[3 * v + 2] = (e[2] * x + e[6] * y + e[10] * z + e[14]) * w;
    const a = N.data[3 * v], b = N.data[3 * v + 1], c = N.data[3 * v + 2];
    const nx = n[0] * a + n[3] * b + n[6] * c, ny = n[1] * a + n[4] * b + n[7] * c, nz = n[2] * a + n[5] * b + n[8] * c;
    let ln = Math.sqrt(nx * nx + ny * ny + nz * nz);
    if (ln === 0) ln = 1;
    const rl = 1 / ln;  // divideScalar(s) = multiplyScalar(1 / s)
    normals[3 * v] = nx * rl;
    normals[3 * v + 1] = ny * rl;
    normals[3 * v + 2] = nz * rl;
  }
  return { positions, normals, uvs: uv, index, material: material(g, prim.material) };
}

/** The default scene's primitives, depth-first, children in glTF order (Structs.ts:118-126). */
function primitives(g) {
  const js = g.json, scene = js.scenes[js.scene || 0], out = [];
  const visit = (ni, parent) => {
    const node = js.nodes[ni];
    const world = multiply(parent, localMatrix(node));  // Object3D.updateMatrixWorld
    if (node.mesh !== undefined) {
      for (const prim of js.meshes[node.mesh].primitives) {
        if ((prim.mode === undefined ? 4 : prim.mode) !== 4) throw new Error('only triangle lists are supported');
        out.push(bake(g, prim, world));
      }
    }
    for (const child of node.children || []) visit(child, world);
  };
  for (const root of scene.nodes) visit(root, [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1]);
  return out;
}

/** mergeGeometries(geoms, true): attributes concatenated, indices offset by the vertices before,
 * one group (first triangle, triangle count) per primitive; uv kept only if every primitive has it. */
function loadGlbGeometry(file) {
  const prims = primitives(readGlb(file));
  const hasUv = prims.every((p) => p.uvs !== null);
  let nv = 0, ni = 0;
  for (const p of prims) { nv += p.positions.length / 3; ni += p.index.length; }
  const positions = new Float32Array(3 * nv), normals = new Float32Array(3 * nv);
  const uvs = hasUv ? new Float32Array(2 * nv) : null, index = new Uint32Array(ni);
  const groups = [], materials = [];
  let vb = 0, ib = 0;
  for (const p of prims) {
    positions.set(p.positions, 3 * vb);
    normals.set(p.normals, 3 * vb);
    if (hasUv) uvs.set(p.uvs, 2 * vb);
    for (let k = 0; k < p.index.length; k++) index[ib + k] = p.index[k] + vb;
    groups.push([ib / 3, p.index.length / 3]);
    vb += p.positions.length / 3;
    ib += p.index.length;
    materials.push(p.material);
  }
  return { positions, normals, uvs, index, groups, materials };
}

module.exports = { readGlb, accessor, primitives, loadGlbGeometry, compose, decompose, localMatrix, multiply, normalMatrix };
