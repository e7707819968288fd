"""Minimal binary-glTF (GLB) reader with the semantics the reference relies on.

The reference loads meshes with three@0.180.0's ``GLTFLoader`` and flattens them in
``Mesh.Load`` (ref: apps/frontend/src/graphics-core/Structs.ts:108-141):

* every ``THREE.Mesh`` reachable from the default scene is visited depth-first
  (``traverseGLTF``, Structs.ts:118-124), multi-primitive glTF meshes become one
  ``THREE.Mesh`` per primitive;
* ``geometry.applyMatrix4(Mesh.matrixWorld)`` bakes the node's world transform into
  positions (``Vector3.applyMatrix4``) and normals (normal matrix, then renormalise),
  computed in f64 and stored back as f32 (Structs.ts:132);
* materials follow GLTFLoader defaults: baseColorFactor (1,1,1), metallic 1,
  roughness 1, emissive (0,0,0), emissiveIntensity 1, ``transparent`` iff
  ``alphaMode == "BLEND"`` (consumed by ``Material``, Structs.ts:311-326).

``three`` itself is not in this container: this is a restatement of
the published loader behaviour, parity with three.js is unpinned.
"""
from __future__ import annotations

import json
import math
import struct
from dataclasses import dataclass, field

import numpy as np

_COMPONENT = {5120: np.int8, 5121: np.uint8, 5122: np.int16, 5123: np.uint16,
              5125: np.uint32, 5126: np.float32}
_NCOMP = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4, "MAT4": 16}


@dataclass
class GltfMaterial:
    """The subset of ``THREE.MeshStandardMaterial`` read by ``Material`` (Structs.ts:311-320)."""
    color: tuple = (1.0, 1.0, 1.0)
    emissive: tuple = (0.0, 0.0, 0.0)
    emissive_intensity: float = 1.0
    metalness: float = 1.0
    roughness: float = 1.0
    transparent: bool = False


@dataclass
class GltfPrimitive:
    positions: np.ndarray            # (V,3) f32, world-space (node transform baked in)
    normals: np.ndarray              # (V,3) f32
    uvs: np.ndarray | None           # (V,2) f32 or None
    indices: np.ndarray              # (3T,) u32
    material: GltfMaterial = field(default_factory=GltfMaterial)


def _compose(t, q, s) -> np.ndarray:
    """three.js Matrix4.compose(position, quaternion, scale): column-major 16 f64, the library's
    own operation order (so the JS host, js/gltf.js, computes the same bits)."""
    x, y, z, w = (float(c) for c in q)
    sx, sy, sz = (float(c) for c in s)
    x2, y2, z2 = x + x, y + y, z + z
    xx, xy, xz = x * x2, x * y2, x * z2
    yy, yz, zz = y * y2, y * z2, z * z2
    wx, wy, wz = w * x2, w * y2, w * z2
    return [(1 - (yy + zz)) * sx, (xy + wz) * sx, (xz - wy) * sx, 0.0,
            (xy - wz) * sy, (1 - (xx + zz)) * sy, (yz + wx) * sy, 0.0,
            (xz + wy) * sz, (yz - wx) * sz, (1 - (xx + yy)) * sz, 0.0,
            float(t[0]), float(t[1]), float(t[2]), 1.0]


def _div(a: float, b: float) -> float:
    """a / b with JavaScript's IEEE semantics (x / 0 = +-Infinity, 0 / 0 = NaN), where Python
    raises: a zero-scale matrix decomposes to the same Infinity / NaN as three.js on the JS host."""
    if b != 0.0:
        return a / b
    if a == 0.0 or math.isnan(a):
        return math.nan
    return math.copysign(math.inf, a) * math.copysign(1.0, b)


def _sqrt(x: float) -> float:
    """Math.sqrt: NaN for a negative argument (Python raises)."""
    return math.sqrt(x) if x >= 0.0 else math.nan


def _decompose(m) -> tuple:
    """three.js Matrix4.decompose(position, quaternion, scale) (f64, the library's order): column
    lengths as scale (the first negated when the determinant is negative), the columns scaled by
    1 / s, Quaternion.setFromRotationMatrix of that 3x3.  A zero-length column gives the JS
    host's Infinity / NaN (never an exception: ADVICE r4), so both hosts bake the same bits."""
    sx = _sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2])
    sy = _sqrt(m[4] * m[4] + m[5] * m[5] + m[6] * m[6])
    sz = _sqrt(m[8] * m[8] + m[9] * m[9] + m[10] * m[10])
    if _determinant(m) < 0:
        sx = -sx
    ix, iy, iz = _div(1.0, sx), _div(1.0, sy), _div(1.0, sz)
    m11, m21, m31 = m[0] * ix, m[1] * ix, m[2] * ix
    m12, m22, m32 = m[4] * iy, m[5] * iy, m[6] * iy
    m13, m23, m33 = m[8] * iz, m[9] * iz, m[10] * iz
    trace = m11 + m22 + m33
    if trace > 0:
        s = _div(0.5, _sqrt(trace + 1.0))
        q = ((m32 - m23) * s, (m13 - m31) * s, (m21 - m12) * s, _div(0.25, s))
    elif m11 > m22 and m11 > m33:
        s = 2.0 * _sqrt(1.0 + m11 - m22 - m33)
        q = (0.25 * s, _div(m12 + m21, s), _div(m13 + m31, s), _div(m32 - m23, s))
    elif m22 > m33:
        s = 2.0 * _sqrt(1.0 + m22 - m11 - m33)
        q = (_div(m12 + m21, s), 0.25 * s, _div(m23 + m32, s), _div(m13 - m31, s))
    else:
        s = 2.0 * _sqrt(1.0 + m33 - m11 - m22)
        q = (_div(m13 + m31, s), _div(m23 + m32, s), 0.25 * s, _div(m21 - m12, s))
    return (m[12], m[13], m[14]), q, (sx, sy, sz)


def _determinant(m) -> float:
    """The 4x4 determinant by cofactors along the first row, as js/gltf.js (only its sign is
    used: decompose's mirrored-scale test)."""
    def a(r, c):
        return m[4 * c + r]

    def det3(r0, r1, r2, c0, c1, c2):
        return (a(r0, c0) * (a(r1, c1) * a(r2, c2) - a(r1, c2) * a(r2, c1))
                - a(r0, c1) * (a(r1, c0) * a(r2, c2) - a(r1, c2) * a(r2, c0))
                + a(r0, c2) * (a(r1, c0) * a(r2, c1) - a(r1, c1) * a(r2, c0)))
    return (a(0, 0) * det3(1, 2, 3, 1, 2, 3) - a(0, 1) * det3(1, 2, 3, 0, 2, 3)
            + a(0, 2) * det3(1, 2, 3, 0, 1, 3) - a(0, 3) * det3(1, 2, 3, 0, 1, 2))


def _node_local_matrix(node) -> list:
    if "matrix" in node:
        # GLTFLoader: node.applyMatrix4(Matrix4.fromArray(matrix)) -- premultiplied onto the
        # node's identity matrix, then DECOMPOSED into position / quaternion / scale, and the
        # world matrix later recomposed from them (Object3D.updateMatrix -> compose): the raw
        # matrix itself is never used.  (Restated from three.js's published source; three is
        # not installed here, so this path is parity-unpinned against the library itself.)
        raw = [float(v) for v in node["matrix"]]
        ident = _compose([0.0, 0.0, 0.0], [0.0, 0.0, 0.0, 1.0], [1.0, 1.0, 1.0])
        t, q, sc = _decompose(_multiply(raw, ident))
        return _compose(t, q, sc)
    return _compose(node.get("translation", [0.0, 0.0, 0.0]), node.get("rotation", [0.0, 0.0, 0.0, 1.0]),
                    node.get("scale", [1.0, 1.0, 1.0]))


def _multiply(a, b) -> list:
    """three.js Matrix4.multiplyMatrices(a, b) (column-major), term order as the library's."""
    out = [0.0] * 16
    for r in range(4):
        for c in range(4):
            out[4 * c + r] = a[r] * b[4 * c] + a[4 + r] * b[4 * c + 1] + a[8 + r] * b[4 * c + 2] + a[12 + r] * b[4 * c + 3]
    return out


def _normal_matrix(m) -> list:
    """three.js Matrix3.getNormalMatrix(m): the upper 3x3, inverted by cofactors, transposed
    (column-major 9 f64); a singular matrix gives zeros."""
    n11, n21, n31 = m[0], m[1], m[2]
    n12, n22, n32 = m[4], m[5], m[6]
    n13, n23, n33 = m[8], m[9], m[10]
    t11 = n33 * n22 - n32 * n23
    t12 = n32 * n13 - n33 * n12
    t13 = n23 * n12 - n22 * n13
    det = n11 * t11 + n21 * t12 + n31 * t13
    if det == 0:
        return [0.0] * 9
    d = 1 / det
    inv = [t11 * d, (n31 * n23 - n33 * n21) * d, (n32 * n21 - n31 * n22) * d,
           t12 * d, (n33 * n11 - n31 * n13) * d, (n31 * n12 - n32 * n11) * d,
           t13 * d, (n21 * n13 - n23 * n11) * d, (n22 * n11 - n21 * n12) * d]
    return [inv[0], inv[3], inv[6], inv[1], inv[4], inv[7], inv[2], inv[5], inv[8]]  # transpose


class Glb:
    def __init__(self, path: str):
        with open(path, "rb") as fh:
            data = fh.read()
        magic, version, length = struct.unpack_from("<III", data, 0)
        if magic != 0x46546C67 or version != 2:
            raise ValueError(f"{path}: not a glTF 2.0 binary")
        off = 12
        self.json = None
        self.bin = b""
        while off < length:
            clen, ctype = struct.unpack_from("<II", data, off)
            chunk = data[off + 8: off + 8 + clen]
            if ctype == 0x4E4F534A:
                self.json = json.loads(chunk)
            elif ctype == 0x004E4942:
                self.bin = chunk
            off += 8 + clen
        if self.json is None:
            raise ValueError(f"{path}: missing JSON chunk")

    def accessor(self, idx: int) -> np.ndarray:
        acc = self.json["accessors"][idx]
        dtype = np.dtype(_COMPONENT[acc["componentType"]])
        ncomp = _NCOMP[acc["type"]]
        count = acc["count"]
        if "bufferView" not in acc:
            return np.zeros((count, ncomp), dtype=dtype)
        bv = self.json["bufferViews"][acc["bufferView"]]
        if bv.get("buffer", 0) != 0:
            raise ValueError("external buffers are not supported")
        start = bv.get("byteOffset", 0) + acc.get("byteOffset", 0)
        stride = bv.get("byteStride", 0) or dtype.itemsize * ncomp
        if stride == dtype.itemsize * ncomp:
            arr = np.frombuffer(self.bin, dtype=dtype, count=count * ncomp, offset=start)
            arr = arr.reshape(count, ncomp)
        else:
            raw = np.frombuffer(self.bin, dtype=np.uint8, count=stride * (count - 1) + dtype.itemsize * ncomp,
                                offset=start)
            arr = np.lib.stride_tricks.as_strided(raw, shape=(count, dtype.itemsize * ncomp),
                                                  strides=(stride, 1)).copy().view(dtype).reshape(count, ncomp)
        if acc.get("normalized", False):
            raise ValueError("normalized accessors are not supported")
        return arr.copy()

    def material(self, idx) -> GltfMaterial:
        if idx is None:
            return GltfMaterial()
        m = self.json["materials"][idx]
        pbr = m.get("pbrMetallicRoughness", {})
        bc = pbr.get("baseColorFactor", [1.0, 1.0, 1.0, 1.0])
        em = m.get("emissiveFactor", [0.0, 0.0, 0.0])
        ext = m.get("extensions", {})
        strength = ext.get("KHR_materials_emissive_strength", {}).get("emissiveStrength", 1.0)
        return GltfMaterial(color=(bc[0], bc[1], bc[2]), emissive=tuple(em), emissive_intensity=strength,
                            metalness=pbr.get("metallicFactor", 1.0), roughness=pbr.get("roughnessFactor", 1.0),
                            transparent=(m.get("alphaMode", "OPAQUE") == "BLEND"))

    def primitives(self) -> list[GltfPrimitive]:
        """Depth-first over the default scene, children in glTF order (Structs.ts:118-126)."""
        js = self.json
        scene = js["scenes"][js.get("scene", 0)]
        out: list[GltfPrimitive] = []

        def visit(node_idx: int, parent):
            node = js["nodes"][node_idx]
            world = _multiply(parent, _node_local_matrix(node))  # Object3D.updateMatrixWorld
            if "mesh" in node:
                for prim in js["meshes"][node["mesh"]]["primitives"]:
                    if prim.get("mode", 4) != 4:
                        raise ValueError("only triangle lists are supported")
                    out.append(self._bake(prim, world))
            for child in node.get("children", []):
                visit(child, world)

        identity = [1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0]
        for root in scene["nodes"]:
            visit(root, identity)
        return out

    def _bake(self, prim, world) -> GltfPrimitive:
        attrs = prim["attributes"]
        pos = self.accessor(attrs["POSITION"]).astype(np.float64)
        nrm = self.accessor(attrs["NORMAL"]).astype(np.float64) if "NORMAL" in attrs else None
        uv = self.accessor(attrs["TEXCOORD_0"]).astype(np.float32) if "TEXCOORD_0" in attrs else None
        if "indices" in prim:
            idx = self.accessor(prim["indices"]).reshape(-1).astype(np.uint32)
        else:
            idx = np.arange(pos.shape[0], dtype=np.uint32)
        e = world
        x, y, z = pos[:, 0], pos[:, 1], pos[:, 2]
        # BufferGeometry.applyMatrix4 -> Vector3.applyMatrix4: w = 1 / (e3 x + e7 y + e11 z + e15),
        # each coordinate (e0 x + e4 y + e8 z + e12) * w, in f64, stored to the f32 attribute
        w = 1 / (e[3] * x + e[7] * y + e[11] * z + e[15])
        p_world = np.stack([(e[0] * x + e[4] * y + e[8] * z + e[12]) * w,
                            (e[1] * x + e[5] * y + e[9] * z + e[13]) * w,
                            (e[2] * x + e[6] * y + e[10] * z + e[14]) * w], axis=1).astype(np.float32)
        if nrm is None:
            raise ValueError("primitives without normals are not supported")
        # BufferAttribute.applyNormalMatrix(Matrix3.getNormalMatrix(m)) -> Vector3.applyMatrix3,
        # then normalize(): divideScalar(length() || 1) = multiplyScalar(1 / len), f64, stored to f32
        n = _normal_matrix(world)
        x, y, z = nrm[:, 0], nrm[:, 1], nrm[:, 2]
        nx = n[0] * x + n[3] * y + n[6] * z
        ny = n[1] * x + n[4] * y + n[7] * z
        nz = n[2] * x + n[5] * y + n[8] * z
        ln = np.sqrt(nx * nx + ny * ny + nz * nz)
        ln = np.where(ln == 0, 1.0, ln)
        rl = 1 / ln
        nrm_w = np.stack([nx * rl, ny * rl, nz * rl], axis=1).astype(np.float32)
        return GltfPrimitive(positions=p_world, normals=nrm_w, uvs=uv, indices=idx,
                             material=self.material(prim.get("material")))
