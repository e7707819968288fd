'use strict';
/**
 * The wgpu-matrix@3.4.0 subset the reference's host uses (Camera.ts, Renderer_TEST.ts:172),
 * with its storage semantics: every function computes in JS numbers (f64) and stores
 * its result into a Float32Array.  The library is not installed here (SURVEY.md §8c);
 * these restate its published formulas and match pathtracerdemo_amd/scene/wgpu_math.py
 * operation for operation, so the Python and JS hosts build bit-identical uniforms.
 */

function out(values) {
  return Float32Array.from(values);
}

const mat4 = {
  identity() {
    return out([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1]);
  },
  translation(v) {
    return out([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, Math.fround(v[0]), Math.fround(v[1]), Math.fround(v[2]), 1]);
  },
  // column-major a * b
  multiply(a, b) {
    const r = new Array(16);
    for (let c = 0; c < 4; c++) {
      for (let row = 0; row < 4; row++) {
        r[c * 4 + row] =
          a[0 * 4 + row] * b[c * 4 + 0] + a[1 * 4 + row] * b[c * 4 + 1] +
          a[2 * 4 + row] * b[c * 4 + 2] + a[3 * 4 + row] * b[c * 4 + 3];
      }
    }
    return out(r);
  },
  // cofactor expansion (2x2 sub-determinants of the top and bottom row pairs)
  invert(m) {
    const [a00, a01, a02, a03, a10, a11, a12, a13, a20, a21, a22, a23, a30, a31, a32, a33] = Array.from(m);
    const b00 = a00 * a11 - a01 * a10, b01 = a00 * a12 - a02 * a10, b02 = a00 * a13 - a03 * a10;
    const b03 = a01 * a12 - a02 * a11, b04 = a01 * a13 - a03 * a11, b05 = a02 * a13 - a03 * a12;
    const b06 = a20 * a31 - a21 * a30, b07 = a20 * a32 - a22 * a30, b08 = a20 * a33 - a23 * a30;
    const b09 = a21 * a32 - a22 * a31, b10 = a21 * a33 - a23 * a31, b11 = a22 * a33 - a23 * a32;
    const det = b00 * b11 - b01 * b10 + b02 * b09 + b03 * b08 - b04 * b07 + b05 * b06;
    const inv = 1.0 / det;
    return out([
      (a11 * b11 - a12 * b10 + a13 * b09) * inv, (a02 * b10 - a01 * b11 - a03 * b09) * inv,
      (a31 * b05 - a32 * b04 + a33 * b03) * inv, (a22 * b04 - a21 * b05 - a23 * b03) * inv,
      (a12 * b08 - a10 * b11 - a13 * b07) * inv, (a00 * b11 - a02 * b08 + a03 * b07) * inv,
      (a32 * b02 - a30 * b05 - a33 * b01) * inv, (a20 * b05 - a22 * b02 + a23 * b01) * inv,
      (a10 * b10 - a11 * b08 + a13 * b06) * inv, (a01 * b08 - a00 * b10 - a03 * b06) * inv,
      (a30 * b04 - a31 * b02 + a33 * b00) * inv, (a21 * b02 - a20 * b04 - a23 * b00) * inv,
      (a11 * b07 - a10 * b09 - a12 * b06) * inv, (a00 * b09 - a01 * b07 + a02 * b06) * inv,
      (a31 * b01 - a30 * b03 - a32 * b00) * inv, (a20 * b03 - a21 * b01 + a22 * b00) * inv,
    ]);
  },
  scaling(v) {
    return out([v[0], 0, 0, 0, 0, v[1], 0, 0, 0, 0, v[2], 0, 0, 0, 0, 1]);
  },
  mul(a, b) { return mat4.multiply(a, b); },
  fromQuat(q) {
    const [x, y, z, w] = Array.from(q);
    const x2 = x + x, y2 = y + y, z2 = z + z;
    const xx = x * x2, yx = y * x2, yy = y * y2;
    const zx = z * x2, zy = z * y2, zz = z * z2;
    const wx = w * x2, wy = w * y2, wz = w * z2;
    return out([1 - yy - zz, yx + wz, zx - wy, 0,
      yx - wz, 1 - xx - zz, zy + wx, 0,
      zx + wy, zy - wx, 1 - xx - yy, 0,
      0, 0, 0, 1]);
  },
  // WebGPU clip space (z in [0, 1])
  perspective(fovy, aspect, near, far) {
    const f = Math.tan(Math.PI * 0.5 - 0.5 * fovy);
    const m = new Array(16).fill(0);
    m[0] = f / aspect;
    m[5] = f;
    m[11] = -1;
    if (Number.isFinite(far)) {
      const rangeInv = 1 / (near - far);
      m[10] = far * rangeInv;
      m[14] = far * near * rangeInv;
    } else {
      m[10] = -1;
      m[14] = -near;
    }
    return out(m);
  },
};

const quat = {
  identity() {
    return out([0, 0, 0, 1]);
  },
  fromAxisAngle(axis, angleInRadians) {
    const halfAngle = angleInRadians * 0.5;
    const s = Math.sin(halfAngle);
    return out([s * axis[0], s * axis[1], s * axis[2], Math.cos(halfAngle)]);
  },
  multiply(a, b) {
    const [ax, ay, az, aw] = Array.from(a);
    const [bx, by, bz, bw] = Array.from(b);
    return out([ax * bw + aw * bx + ay * bz - az * by,
      ay * bw + aw * by + az * bx - ax * bz,
      az * bw + aw * bz + ax * by - ay * bx,
      aw * bw - ax * bx - ay * by - az * bz]);
  },
  fromEuler(x, y, z, order) {
    if (order !== 'yxz') throw new Error(`quat.fromEuler: order ${order} not supported`);
    const sx = Math.sin(x * 0.5), cx = Math.cos(x * 0.5);
    const sy = Math.sin(y * 0.5), cy = Math.cos(y * 0.5);
    const sz = Math.sin(z * 0.5), cz = Math.cos(z * 0.5);
    return out([sx * cy * cz + cx * sy * sz, cx * sy * cz - sx * cy * sz,
      cx * cy * sz - sx * sy * cz, cx * cy * cz + sx * sy * sz]);
  },
};

const vec3 = {
  fromValues(x, y, z) {
    return out([x, y, z]);
  },
  create(x = 0, y = 0, z = 0) {
    return out([x, y, z]);
  },
  scale(v, k) {
    return out([v[0] * k, v[1] * k, v[2] * k]);
  },
  dot(a, b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
  },
  cross(a, b) {
    return out([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]);
  },
  len(v) {
    return Math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  },
  length(v) {
    return Math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  },
  normalize(v) {
    const l = Math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    return l > 0.00001 ? out([v[0] / l, v[1] / l, v[2] / l]) : out([0, 0, 0]);
  },
  // a + b * scale, into dst when given (InputController.ts:92-110 accumulates in place)
  addScaled(a, b, scale, dst) {
    const r = [a[0] + b[0] * scale, a[1] + b[1] * scale, a[2] + b[2] * scale];
    if (!dst) return out(r);
    dst[0] = r[0]; dst[1] = r[1]; dst[2] = r[2];
    return dst;
  },
  // v rotated by the unit quaternion q: v + 2w (q.xyz x v) + 2 q.xyz x (q.xyz x v)  (Camera.ts:71)
  transformQuat(v, q) {
    const qx = q[0], qy = q[1], qz = q[2], w2 = q[3] * 2;
    const x = v[0], y = v[1], z = v[2];
    const uvX = qy * z - qz * y, uvY = qz * x - qx * z, uvZ = qx * y - qy * x;
    return out([x + uvX * w2 + (qy * uvZ - qz * uvY) * 2,
      y + uvY * w2 + (qz * uvX - qx * uvZ) * 2,
      z + uvZ * w2 + (qx * uvY - qy * uvX) * 2]);
  },
};

const vec4 = {
  create(x = 0, y = 0, z = 0, w = 0) {
    return out([x, y, z, w]);
  },
};

module.exports = { mat4, quat, vec3, vec4 };
