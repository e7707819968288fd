"""Host-side matrix / quaternion helpers with wgpu-matrix@3.4.0 storage semantics.

wgpu-matrix computes every function in JS numbers (f64) and stores its result into a
``Float32Array``; the reference chains these (Camera.ts:47-64,165-168;
Structs.ts:27-38; World.ts:14-33; Renderer_TEST.ts:172), so each function below
computes in float64 and rounds its *output* to float32.  The library itself is not
in this container: the formulas restate its published source; the
kernels never depend on them because the boundary receives the finished f32 arrays.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32


def _out(m) -> np.ndarray:
    return np.asarray(m, dtype=np.float64).astype(np.float32)


def mat4_identity() -> np.ndarray:
    return np.eye(4, dtype=np.float32).reshape(-1)


def mat4_translation(v) -> np.ndarray:
    m = np.eye(4, dtype=np.float64).reshape(-1)
    m[12:15] = np.asarray(v, dtype=np.float32)
    return _out(m)


def mat4_scaling(v) -> np.ndarray:
    v = np.asarray(v, dtype=np.float32).astype(np.float64)
    m = np.zeros(16)
    m[0], m[5], m[10], m[15] = v[0], v[1], v[2], 1.0
    return _out(m)


def mat4_multiply(a, b) -> np.ndarray:
    """Column-major a*b (wgpu-matrix mat4.multiply); left-to-right f64 sums, as the JS host
    (pathtracerdemo_amd/js/wgpu_math.js) computes them."""
    a = [float(v) for v in np.asarray(a, dtype=np.float32)]
    b = [float(v) for v in np.asarray(b, dtype=np.float32)]
    r = [0.0] * 16
    for c in range(4):
        for row in range(4):
            r[c * 4 + row] = (a[row] * b[c * 4] + a[4 + row] * b[c * 4 + 1]
                              + a[8 + row] * b[c * 4 + 2] + a[12 + row] * b[c * 4 + 3])
    return _out(r)


def mat4_invert(m) -> np.ndarray:
    """wgpu-matrix mat4.invert: cofactor expansion over 2x2 sub-determinants, f64."""
    (a00, a01, a02, a03, a10, a11, a12, a13,
     a20, a21, a22, a23, a30, a31, a32, a33) = (float(v) for v in np.asarray(m, dtype=np.float32))
    b00, b01, b02 = a00 * a11 - a01 * a10, a00 * a12 - a02 * a10, a00 * a13 - a03 * a10
    b03, b04, b05 = a01 * a12 - a02 * a11, a01 * a13 - a03 * a11, a02 * a13 - a03 * a12
    b06, b07, b08 = a20 * a31 - a21 * a30, a20 * a32 - a22 * a30, a20 * a33 - a23 * a30
    b09, b10, b11 = a21 * a32 - a22 * a31, a21 * a33 - a23 * a31, a22 * a33 - a23 * a32
    det = b00 * b11 - b01 * b10 + b02 * b09 + b03 * b08 - b04 * b07 + b05 * b06
    inv = 1.0 / det
    return _out([
        (a11 * b11 - a12 * b10 + a13 * b09) * inv, (a02 * b10 - a01 * b11 - a03 * b09) * inv,
        (a31 * b05 - a32 * b04 + a33 * b03) * inv, (a22 * b04 - a21 * b05 - a23 * b03) * inv,
        (a12 * b08 - a10 * b11 - a13 * b07) * inv, (a00 * b11 - a02 * b08 + a03 * b07) * inv,
        (a32 * b02 - a30 * b05 - a33 * b01) * inv, (a20 * b05 - a22 * b02 + a23 * b01) * inv,
        (a10 * b10 - a11 * b08 + a13 * b06) * inv, (a01 * b08 - a00 * b10 - a03 * b06) * inv,
        (a30 * b04 - a31 * b02 + a33 * b00) * inv, (a21 * b02 - a20 * b04 - a23 * b00) * inv,
        (a11 * b07 - a10 * b09 - a12 * b06) * inv, (a00 * b09 - a01 * b07 + a02 * b06) * inv,
        (a31 * b01 - a30 * b03 - a32 * b00) * inv, (a20 * b03 - a21 * b01 + a22 * b00) * inv,
    ])


def mat4_from_quat(q) -> np.ndarray:
    x, y, z, w = (float(c) for c in np.asarray(q, dtype=np.float32))
    x2, y2, z2 = x + x, y + y, z + z
    xx, yx, yy = x * x2, y * x2, y * y2
    zx, zy, zz = z * x2, z * y2, z * z2
    wx, wy, wz = w * x2, w * y2, w * z2
    return _out([1 - yy - zz, yx + wz, zx - wy, 0,
                 yx - wz, 1 - xx - zz, zy + wx, 0,
                 zx + wy, zy - wx, 1 - xx - yy, 0,
                 0, 0, 0, 1])


def mat4_perspective(fovy: float, aspect: float, near: float, far: float) -> np.ndarray:
    """WebGPU clip space (z in [0,1]) perspective, as wgpu-matrix mat4.perspective."""
    f = math.tan(math.pi * 0.5 - 0.5 * fovy)
    m = [0.0] * 16
    m[0] = f / aspect
    m[5] = f
    m[11] = -1.0
    if math.isfinite(far):
        range_inv = 1.0 / (near - far)
        m[10] = far * range_inv
        m[14] = far * near * range_inv
    else:
        m[10] = -1.0
        m[14] = -near
    return _out(m)


def quat_identity() -> np.ndarray:
    return np.array([0, 0, 0, 1], dtype=np.float32)


def quat_from_axis_angle(axis, angle: float) -> np.ndarray:
    axis = np.asarray(axis, dtype=np.float32).astype(np.float64)
    half = angle * 0.5
    s = math.sin(half)
    return _out([s * axis[0], s * axis[1], s * axis[2], math.cos(half)])


def quat_multiply(a, b) -> np.ndarray:
    ax, ay, az, aw = (float(c) for c in np.asarray(a, dtype=np.float32))
    bx, by, bz, bw = (float(c) for c in np.asarray(b, dtype=np.float32))
    return _out([ax * bw + aw * bx + ay * bz - az * by,
                 ay * bw + aw * by + az * bx - ax * bz,
                 az * bw + aw * bz + ax * by - ay * bx,
                 aw * bw - ax * bx - ay * by - az * bz])


def quat_from_euler(x: float, y: float, z: float, order: str) -> np.ndarray:
    sx, cx = math.sin(x * 0.5), math.cos(x * 0.5)
    sy, cy = math.sin(y * 0.5), math.cos(y * 0.5)
    sz, cz = math.sin(z * 0.5), math.cos(z * 0.5)
    if order != "yxz":
        raise NotImplementedError(order)
    return _out([sx * cy * cz + cx * sy * sz,
                 cx * sy * cz - sx * cy * sz,
                 cx * cy * sz - sx * sy * cz,
                 cx * cy * cz + sx * sy * sz])


def vec3_normalize(v) -> np.ndarray:
    v = np.asarray(v, dtype=np.float32).astype(np.float64)
    ln = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    if ln > 0.00001:
        return _out(v / ln)
    return np.zeros(3, dtype=np.float32)


def vec3_cross(a, b) -> np.ndarray:
    a = np.asarray(a, dtype=np.float32).astype(np.float64)
    b = np.asarray(b, dtype=np.float32).astype(np.float64)
    return _out([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]])


def vec3_len(v) -> float:
    v = np.asarray(v, dtype=np.float32).astype(np.float64)
    return math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])


def vec3_add_scaled(a, b, scale: float) -> np.ndarray:
    """wgpu-matrix vec3.addScaled: a + b * scale (InputController.ts:92-110)."""
    a = np.asarray(a, dtype=np.float32).astype(np.float64)
    b = np.asarray(b, dtype=np.float32).astype(np.float64)
    return _out([a[0] + b[0] * scale, a[1] + b[1] * scale, a[2] + b[2] * scale])


def vec3_transform_quat(v, q) -> np.ndarray:
    """wgpu-matrix vec3.transformQuat: v + 2w (q.xyz x v) + 2 q.xyz x (q.xyz x v) (Camera.ts:71)."""
    x, y, z = (float(c) for c in np.asarray(v, dtype=np.float32))
    qx, qy, qz, qw = (float(c) for c in np.asarray(q, dtype=np.float32))
    w2 = qw * 2
    ux, uy, uz = qy * z - qz * y, qz * x - qx * z, qx * y - qy * x
    return _out([x + ux * w2 + (qy * uz - qz * uy) * 2,
                 y + uy * w2 + (qz * ux - qx * uz) * 2,
                 z + uz * w2 + (qx * uy - qy * ux) * 2])
