"""Scene model and serialisation into the reference's three flat u32 buffers.

Restates, in numpy, the reference's host-side scene compile:

* ``Instance`` (Structs.ts:9-56): ``M = I·S·R·T`` (sic, the reference's order),
  ``M⁻¹``, 33 words per instance;
* ``Mesh.Load`` / ``Mesh.Serialize`` (Structs.ts:108-215): merge primitives with one
  group per primitive, one BLAS root per group, vertices 8 words (pos, normal, uv);
* ``Material`` 15 words, ``Light`` 18 words and its subclasses (Structs.ts:294-486);
* ``World.LoadFromScene`` / ``PackWorldData`` / ``GetLightCDFBuffer``
  (World.ts:14-33,118-231);
* ``Renderer.SerializeWorldData`` (Renderer_TEST.ts:267-420) and the 33-word uniform
  block of ``Renderer.Update`` (Renderer_TEST.ts:165-206).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass

import numpy as np

from . import wgpu_math as wm
from .bvh import build_blas
from .gltf import Glb

STRIDE_INSTANCE = 33
STRIDE_DESCRIPTOR = 6
STRIDE_MATERIAL = 15
STRIDE_LIGHT = 18
STRIDE_VERTEX = 8
UNIFORM_WORDS = 33

LIGHT_DIRECTION, LIGHT_POINT, LIGHT_RECT = 0, 1, 2

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                         "scenes", "assets")
SCENE_DIR = os.path.dirname(ASSET_DIR)


def merge_arrays(arrays):
    """ResourceManager.MergeArrays (ResourceManager.ts:23-43): concat + element offsets."""
    if not arrays:
        return np.zeros(0, dtype=np.uint32), np.zeros(0, dtype=np.uint32)
    offsets = np.zeros(len(arrays), dtype=np.uint32)
    for i in range(len(arrays) - 1):
        offsets[i + 1] = offsets[i] + len(arrays[i])
    merged = np.concatenate([np.asarray(a, dtype=np.uint32).reshape(-1) for a in arrays]) \
        if any(len(a) for a in arrays) else np.zeros(0, dtype=np.uint32)
    return merged.astype(np.uint32), offsets


# --------------------------------------------------------------------------- instances
class Instance:
    """Structs.ts:9-56."""

    def __init__(self, mesh_id: str, translation=(0, 0, 0), rotation=None, scale=(1, 1, 1)):
        self.mesh_id = mesh_id
        t = wm.mat4_translation(np.asarray(translation, dtype=np.float32))
        r = wm.mat4_from_quat(wm.quat_identity() if rotation is None else rotation)
        s = wm.mat4_scaling(np.asarray(scale, dtype=np.float32))
        m = wm.mat4_identity()
        m = wm.mat4_multiply(m, s)
        m = wm.mat4_multiply(m, r)
        m = wm.mat4_multiply(m, t)
        self.model = m
        self.model_inv = wm.mat4_invert(m)

    def serialize(self, mesh_index: dict) -> np.ndarray:
        out = np.zeros(STRIDE_INSTANCE, dtype=np.uint32)
        out[0:16] = self.model.view(np.uint32)
        out[16:32] = self.model_inv.view(np.uint32)
        out[32] = mesh_index[self.mesh_id]
        return out


# --------------------------------------------------------------------------- materials
def serialize_material(mat) -> np.ndarray:
    """Material constructor + Serialize (Structs.ts:311-346): albedo alpha is 1.0,
    transmission = transparent ? 1 : 0, IOR fixed 1.5, words 12..14 unused (0)."""
    f = np.zeros(STRIDE_MATERIAL, dtype=np.float32)
    f[0:3] = mat.color
    f[3] = 1.0
    f[4:7] = mat.emissive
    f[7] = mat.emissive_intensity
    f[8] = mat.metalness
    f[9] = mat.roughness
    f[10] = 1.0 if mat.transparent else 0.0
    f[11] = 1.5
    return f.view(np.uint32)


# --------------------------------------------------------------------------- meshes
@dataclass
class SerializedMesh:
    blas: np.ndarray
    sub_blas_roots: np.ndarray
    vertices: np.ndarray
    indices: np.ndarray
    materials: np.ndarray
    max_depth: int


@dataclass
class MeshData:
    """What the reference's Mesh constructor keeps (Structs.ts:58-106): the merged geometry
    after three-mesh-bvh reordered its index buffer, one BLAS root (node array) per group /
    sub-mesh, and the materials.  `Mesh.Serialize` (Structs.ts:143-215) flattens it; the
    Node host restates that step from an export of this state (export.export_meshes)."""
    positions: np.ndarray        # (V, 3) f32
    normals: np.ndarray          # (V, 3) f32
    uvs: np.ndarray | None       # (V, 2) f32, or None when a primitive has no UVs
    indices: np.ndarray          # (3T,) u32, BVH-reordered
    roots: list                  # per sub-mesh: u32 node array (8 words per node)
    materials: list              # GltfMaterial per sub-mesh
    max_depth: int


_MESH_CACHE: dict = {}
_DATA_CACHE: dict = {}


def mesh_data(name: str, asset_dir: str | None = None) -> MeshData:
    """Mesh.Load + constructor (Structs.ts:71-141): GLB primitives merged with one group
    per primitive (mergeGeometries(geoms, true)), SAH BLAS per group."""
    path = os.path.join(asset_dir or ASSET_DIR, name + ".glb")
    key = (os.path.abspath(path), os.path.getmtime(path))
    if key in _DATA_CACHE:
        return _DATA_CACHE[key]
    prims = Glb(path).primitives()
    has_uv = all(p.uvs is not None for p in prims)
    pos, nrm, uvs, idx, groups, mats = [], [], [], [], [], []
    vbase = 0
    ibase = 0
    for p in prims:               # mergeGeometries(geoms, useGroups=true)
        pos.append(p.positions)
        nrm.append(p.normals)
        if has_uv:
            uvs.append(p.uvs)
        idx.append(p.indices.astype(np.uint64) + vbase)
        groups.append((ibase // 3, len(p.indices) // 3))
        vbase += p.positions.shape[0]
        ibase += len(p.indices)
        mats.append(p.material)
    positions = np.concatenate(pos).astype(np.float32)
    normals = np.concatenate(nrm).astype(np.float32)
    indices = np.concatenate(idx).astype(np.uint32)
    roots, indices, max_depth = build_blas(positions, indices, groups)
    md = MeshData(positions=positions, normals=normals,
                  uvs=np.concatenate(uvs).astype(np.float32) if has_uv else None, indices=indices,
                  roots=[np.asarray(r, dtype=np.uint32) for r in roots], materials=mats, max_depth=max_depth)
    _DATA_CACHE[key] = md
    return md


def load_mesh(name: str, asset_dir: str | None = None) -> SerializedMesh:
    """Mesh.Load + constructor + Serialize (Structs.ts:71-215)."""
    path = os.path.join(asset_dir or ASSET_DIR, name + ".glb")
    key = (os.path.abspath(path), os.path.getmtime(path))
    if key in _MESH_CACHE:
        return _MESH_CACHE[key]
    md = mesh_data(name, asset_dir)
    blas, root_offsets = merge_arrays(md.roots)
    vert = np.zeros((md.positions.shape[0], STRIDE_VERTEX), dtype=np.float32)
    vert[:, 0:3] = md.positions
    vert[:, 3:6] = md.normals
    if md.uvs is not None:
        vert[:, 6:8] = md.uvs
    sm = SerializedMesh(blas=blas, sub_blas_roots=root_offsets,
                        vertices=vert.reshape(-1).view(np.uint32), indices=md.indices,
                        materials=merge_arrays([serialize_material(m) for m in md.materials])[0],
                        max_depth=md.max_depth)
    _MESH_CACHE[key] = sm
    return sm


# --------------------------------------------------------------------------- lights
class Light:
    """Structs.ts:349-486 (directional / point / rect)."""

    def __init__(self, position, direction, color, u, v, light_type: int, intensity: float, area: float):
        self.position = np.asarray(position, dtype=np.float32)
        self.direction = np.asarray(direction, dtype=np.float32)
        self.color = np.asarray(color, dtype=np.float32)
        self.u = np.asarray(u, dtype=np.float32)
        self.v = np.asarray(v, dtype=np.float32)
        self.light_type = int(light_type)
        self.intensity = float(intensity)
        self.area = float(area)

    @staticmethod
    def directional(direction, color, intensity):
        z = np.zeros(3, np.float32)
        return Light(z, direction, color, z, z, LIGHT_DIRECTION, intensity, 0.0)

    @staticmethod
    def point(position, color, intensity):
        z = np.zeros(3, np.float32)
        return Light(position, z, color, z, z, LIGHT_POINT, intensity, 0.0)

    @staticmethod
    def rect(position, color, u, v, intensity):
        direction = wm.vec3_normalize(wm.vec3_cross(u, v))
        area = 4.0 * wm.vec3_len(u) * wm.vec3_len(v)
        return Light(position, direction, color, u, v, LIGHT_RECT, intensity, area)

    def luminance(self) -> float:
        """GetLuminance (Structs.ts:385-389): vec3.scale and vec3.fromValues store f32, so
        both the scaled colour and the Rec. 709 weights are f32; vec3.dot sums in f64."""
        c = (self.color.astype(np.float64) * self.intensity).astype(np.float32).astype(np.float64)
        w = np.array([0.2126, 0.7152, 0.0722], dtype=np.float32).astype(np.float64)
        return float(c[0] * w[0] + c[1] * w[1] + c[2] * w[2])

    def serialize(self) -> np.ndarray:
        f = np.zeros(STRIDE_LIGHT, dtype=np.float32)
        f[0:3] = self.position
        f[3:6] = self.direction
        f[6:9] = self.color
        f[9:12] = self.u
        f[12:15] = self.v
        f[16] = self.intensity
        f[17] = self.area
        out = f.view(np.uint32).copy()
        out[15] = self.light_type
        return out


def euler_degrees_to_quat(e) -> np.ndarray:
    """World.ts:14-33: q = qz · (qy · qx)."""
    d2r = math.pi / 180.0
    x, y, z = (float(c) * d2r for c in e)  # the Scene JSON's numbers, not f32-rounded
    qx = wm.quat_from_axis_angle((1, 0, 0), x)
    qy = wm.quat_from_axis_angle((0, 1, 0), y)
    qz = wm.quat_from_axis_angle((0, 0, 1), z)
    r = wm.quat_multiply(qy, qx)
    return wm.quat_multiply(qz, r)


# --------------------------------------------------------------------------- world
class World:
    """World.ts:36-231."""

    def __init__(self, asset_dir: str | None = None):
        self.instances: dict[str, Instance] = {}
        self.lights: list[Light] = []
        self.asset_dir = asset_dir

    def add_instance(self, name, mesh_name, translation=(0, 0, 0), rotation=None, scale=(1, 1, 1)):
        self.instances[name] = Instance(mesh_name, translation, rotation, scale)

    def load_from_scene(self, scene: dict) -> "World":
        self.instances = {}
        self.lights = []
        for asset in scene["assets"]:
            t = asset["type"]
            if t == "object":
                if not asset.get("meshName") or not asset.get("transform"):
                    continue
                tr = asset["transform"]
                self.add_instance(asset["id"], asset["meshName"], tr["position"],
                                  euler_degrees_to_quat(tr["rotation"]), tr["scale"])
            elif t == "directional-light":
                p = asset.get("lightParams")
                if not p:
                    continue
                self.lights.append(Light.directional(wm.vec3_normalize(p["direction"]), p["color"], p["intensity"]))
            elif t == "point-light":
                p = asset.get("lightParams")
                if not p:
                    continue
                self.lights.append(Light.point(p["position"], p["color"], p["intensity"]))
            elif t == "rect-light":
                p = asset.get("lightParams")
                if not p:
                    continue
                self.lights.append(Light.rect(p["position"], p["color"], p["u"], p["v"], p["intensity"]))
        return self

    def pack(self):
        """PackWorldData (World.ts:184-212): meshes in first-use order."""
        inst = list(self.instances.values())
        used: dict[str, SerializedMesh] = {}
        for i in inst:
            used[i.mesh_id] = load_mesh(i.mesh_id, self.asset_dir)
        mesh_index = {name: k for k, name in enumerate(used.keys())}
        return inst, list(used.values()), mesh_index

    def light_cdf(self) -> np.ndarray:
        """GetLightCDFBuffer (World.ts:214-231), f32 storage with f64 arithmetic."""
        n = len(self.lights)
        lum = np.array([l.luminance() for l in self.lights], dtype=np.float32)
        s = 0.0
        for i in range(n):
            s += float(lum[i])
        for i in range(n):
            lum[i] = np.float32(float(lum[i]) / s)
        for i in range(1, n):
            lum[i] = np.float32(float(lum[i]) + float(lum[i - 1]))
        if n:
            lum[n - 1] = 1.0
        return lum.view(np.uint32)


@dataclass
class CompiledScene:
    """The reference's device inputs: SceneBuffer, GeometryBuffer, AccelBuffer + offsets."""
    scene: np.ndarray
    geometry: np.ndarray
    accel: np.ndarray
    offsets: dict
    instance_count: int
    light_count: int
    max_bvh_depth: int
    triangle_count: int

    def uniform(self, width: int, height: int, vp_inv: np.ndarray, cam_pos, frame_index: int) -> np.ndarray:
        """The 33-word uniform block (Renderer_TEST.ts:174-202)."""
        u = np.zeros(UNIFORM_WORDS, dtype=np.uint32)
        u[0], u[1], u[2], u[3] = width, height, 10, 1
        u[4:20] = np.asarray(vp_inv, dtype=np.float32).view(np.uint32)
        u[20:23] = np.asarray(cam_pos, dtype=np.float32).view(np.uint32)
        u[23] = frame_index
        o = self.offsets
        u[24:31] = [o["mesh_descriptor"], o["material"], o["light"], o["lights_cdf"], o["index"],
                    o["sub_blas_root"], o["blas"]]
        u[31] = self.instance_count
        u[32] = self.light_count
        return u


def serialize_world(world: World) -> CompiledScene:
    """Renderer_TEST.SerializeWorldData (Renderer_TEST.ts:267-420)."""
    inst, meshes, mesh_index = world.pack()
    instance_raw = merge_arrays([i.serialize(mesh_index) for i in inst])[0]
    light_raw = merge_arrays([l.serialize() for l in world.lights])[0]
    cdf_raw = world.light_cdf()
    vert_raw, vert_off = merge_arrays([m.vertices for m in meshes])
    idx_raw, idx_off = merge_arrays([m.indices for m in meshes])
    mat_raw, mat_off = merge_arrays([m.materials for m in meshes])
    root_raw, root_off = merge_arrays([m.sub_blas_roots for m in meshes])
    blas_raw, blas_off = merge_arrays([m.blas for m in meshes])
    descs = []
    for k, m in enumerate(meshes):
        descs.append(np.array([vert_off[k], idx_off[k], mat_off[k], root_off[k], blas_off[k],
                               len(m.sub_blas_roots)], dtype=np.uint32))
    desc_raw = merge_arrays(descs)[0]
    scene, so = merge_arrays([instance_raw, desc_raw, mat_raw, light_raw, cdf_raw])
    geometry, go = merge_arrays([vert_raw, idx_raw, root_raw])
    accel, ao = merge_arrays([np.zeros(0, np.uint32), blas_raw])
    offsets = dict(mesh_descriptor=int(so[1]), material=int(so[2]), light=int(so[3]), lights_cdf=int(so[4]),
                   index=int(go[1]), sub_blas_root=int(go[2]), blas=int(ao[1]))
    return CompiledScene(scene=scene, geometry=geometry, accel=accel, offsets=offsets,
                         instance_count=len(inst), light_count=len(world.lights),
                         max_bvh_depth=max((m.max_depth for m in meshes), default=0),
                         triangle_count=sum(len(m.indices) // 3 for m in meshes))


def load_scene_json(name: str) -> dict:
    with open(os.path.join(SCENE_DIR, name + ".json")) as fh:
        return json.load(fh)


def scene_from_backend(record) -> dict:
    """A Scene from the backend's record: SceneResponse carries `assets` as a JSON string
    (apps/backend/.../dto/SceneResponse.java:24-25, stored as jsonb by entity/Scene.java:39-41);
    the frontend's Scene type (GC/Structs.ts:541-556) wants the array.  Accepts the record as a
    JSON string or dict, with `assets` as a string or already parsed."""
    rec = json.loads(record) if isinstance(record, (str, bytes)) else dict(record)
    assets = json.loads(rec["assets"]) if isinstance(rec.get("assets"), (str, bytes)) else rec.get("assets")
    if not isinstance(assets, list):
        raise ValueError("scene assets must be an array (or its JSON string)")
    rec["assets"] = assets
    return rec


def compile_scene(name_or_dict, asset_dir: str | None = None) -> CompiledScene:
    """A scene name (scenes/<name>.json), a Scene dict, or a backend record (scene_from_backend)."""
    if isinstance(name_or_dict, str) and not name_or_dict.lstrip().startswith("{"):
        scene = load_scene_json(name_or_dict)
    else:
        scene = scene_from_backend(name_or_dict)
    return serialize_world(World(asset_dir).load_from_scene(scene))
