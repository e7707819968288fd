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


def _quat_to_mat(q):
    x, y, z, w = (float(c) for c in q)
    # three.js Matrix4.compose (f64)
    x2, y2, z2 = x + x, y + y, z + z
    xx, xy, xz = x * x2, x * y2, x * z2
    yy, yz, zz = y * y2, y * z2, z * z2
    wx, wy, wz = w * x2, w * y2, w * z2
    return np.array([[1 - (yy + zz), xy - wz, xz + wy],
                     [xy + wz, 1 - (xx + zz), yz - wx],
                     [xz - wy, yz + wx, 1 - (xx + yy)]], dtype=np.float64)


def _node_local_matrix(node) -> np.ndarray:
    if "matrix" in node:
        return np.array(node["matrix"], dtype=np.float64).reshape(4, 4).T  # column-major in glTF
    t = node.get("translation", [0.0, 0.0, 0.0])
    r = node.get("rotation", [0.0, 0.0, 0.0, 1.0])
    s = node.get("scale", [1.0, 1.0, 1.0])
    m = np.eye(4, dtype=np.float64)
    rot = _quat_to_mat(r)
    m[:3, :3] = rot * np.array(s, dtype=np.float64)[None, :]
    m[:3, 3] = t
    return m


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

        def visit(node_idx: int, parent: np.ndarray):
            node = js["nodes"][node_idx]
            world = parent @ _node_local_matrix(node)
            if "mesh" in node:
                for prim in js["meshes"][node["mesh"]]["primitives"]:
                    if prim.get("mode", 4) != 4:
                        raise ValueError("only triangle lists are supported")
                    out.append(self._bake(prim, world))
            for child in node.get("children", []):
                visit(child, world)

        for root in scene["nodes"]:
            visit(root, np.eye(4, dtype=np.float64))
        return out

    def _bake(self, prim, world: np.ndarray) -> GltfPrimitive:
        attrs = prim["attributes"]
        pos = self.accessor(attrs["POSITION"]).astype(np.float64)
        nrm = self.accessor(attrs["NORMAL"]).astype(np.float64) if "NORMAL" in attrs else None
        uv = self.accessor(attrs["TEXCOORD_0"]).astype(np.float32) if "TEXCOORD_0" in attrs else None
        if "indices" in prim:
            idx = self.accessor(prim["indices"]).reshape(-1).astype(np.uint32)
        else:
            idx = np.arange(pos.shape[0], dtype=np.uint32)
        # Vector3.applyMatrix4 (with the projective w, exactly 1 for affine nodes)
        h = np.concatenate([pos, np.ones((pos.shape[0], 1))], axis=1) @ world.T
        p_world = (h[:, :3] / h[:, 3:4]).astype(np.float32)
        if nrm is None:
            raise ValueError("primitives without normals are not supported")
        # BufferAttribute.applyNormalMatrix: Matrix3.getNormalMatrix = inverse-transpose, then normalize()
        nm = np.linalg.inv(world[:3, :3]).T
        n = nrm @ nm.T
        ln = np.sqrt((n * n).sum(axis=1, keepdims=True))
        n = np.where(ln > 0, n / np.where(ln > 0, ln, 1.0), 0.0).astype(np.float32)
        return GltfPrimitive(positions=p_world, normals=n, uvs=uv, indices=idx,
                             material=self.material(prim.get("material")))
