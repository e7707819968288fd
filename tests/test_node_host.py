"""The Node host (north_star: "the TypeScript host calls a thin Node N-API C-ABI addon"):
pathtracerdemo_amd/js/{ptx_node.c, NativeRenderer.js, Camera.js, wgpu_math.js}.

CPU: the addon loads and exports the whole C ABI surface; NativeRenderer builds the same
33-word uniform block as the Python host for several camera poses (bit for bit).
GPU: frames rendered through NativeRenderer (Update + RenderAsync, WebGPUEngine's loop)
are bit-identical to the CPU oracle.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import uniform_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
ADDON = os.path.join(ROOT, "pathtracerdemo_amd", "ptx_node.node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")

EXPORTS = ["abiVersion", "create", "uploadScene", "setFrame", "render", "renderAsync", "runPass", "runPasses",
           "resetAccumulation", "synchronize", "getStats", "resetStats", "readBuffer", "writeBuffer",
           "trace", "destroy", "lastError", "renderBands", "renderBandsAsync", "commUniqueId", "commInit",
           "commInitAll", "rowCensus", "present", "presentAsync", "presentPoll", "buildInfo"]


@pytest.fixture(scope="module")
def scene_dir(scene1, tmp_path_factory):
    from pathtracerdemo_amd.scene.export import export_compiled
    return export_compiled(scene1, str(tmp_path_factory.mktemp("c1")), "dummy_scene_1")


def node(script, *args, stdin=None, timeout=300):
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", script), *args], input=stdin,
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    return p.stdout


def test_addon_exports_the_abi():
    assert os.path.exists(ADDON), "build it: make -C pathtracerdemo_amd/js (or __graft_entry__.build())"
    out = subprocess.run([NODE, "-e", f"const a=require({json.dumps(ADDON)});"
                          "process.stdout.write(JSON.stringify([Object.keys(a), a.abiVersion()]))"],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    keys, abi = json.loads(out.stdout)
    assert sorted(keys) == sorted(EXPORTS)
    assert abi == 5


def test_js_uniform_matches_python_host(scene1, scene_dir):
    from pathtracerdemo_amd.scene.camera import Camera
    poses = [{"loc": [0, 0, 6], "yaw": 0, "pitch": 0, "frame": 1},
             {"loc": [0.5, -0.25, 4.0], "yaw": 37, "pitch": -12, "frame": 7},
             {"loc": [-1, 1.5, 3], "yaw": -400, "pitch": 200, "frame": 123456}]
    W, H = 320, 180
    got = json.loads(node("uniform_dump.js", stdin=json.dumps(
        {"sceneDir": scene_dir, "width": W, "height": H, "poses": poses})))
    for p, g in zip(poses, got):
        cam = Camera(W, H)
        cam.set_location(*p["loc"])
        cam.set_yaw(p["yaw"])
        cam.set_pitch(p["pitch"])
        ref = scene1.uniform(W, H, cam.view_projection_inverse(), cam.location, p["frame"])
        np.testing.assert_array_equal(np.array(g, dtype=np.uint64).astype(np.uint32), ref)


CANVASES = [[600, 450, 0], [96, 64, 1], [1920, 1080, 0], [257, 131, 1]]


def test_js_present_image_matches_the_render_pass_restatement(oracle_mod, tmp_path):
    """presentImage (the reference's render pass on the host, for frames gathered from bands):
    the 600 x 450 texel window of FragmentShader.wgsl through VertexShader.wgsl's quad onto
    canvases of several sizes, unorm8 RGBA / BGRA -- equal byte for byte to oracle.present,
    including out-of-range values (negative, > 1, NaN, inf) and texels outside a small image."""
    rng = np.random.default_rng(3)
    for W, H in ((640, 480), (300, 200)):
        img = rng.uniform(-0.2, 1.2, size=(H, W, 4)).astype(np.float32)
        img.reshape(-1)[rng.integers(0, img.size, 64)] = np.nan
        img.reshape(-1)[rng.integers(0, img.size, 16)] = np.inf
        img[::7, ::5, :3] = np.float32(0.5) / np.float32(255.0) + np.float32(0.0)  # near half-way cases
        f = str(tmp_path / f"img{W}.f32")
        img.tofile(f)
        node("present_host.js", json.dumps({"img": f, "width": W, "height": H, "canvases": CANVASES, "out": f}))
        for i, (cw, ch, bgra) in enumerate(CANVASES):
            got = np.fromfile(f"{f}.{i}", dtype=np.uint8).reshape(ch, cw, 4)
            np.testing.assert_array_equal(got, oracle_mod.present(img, cw, ch, bool(bgra)), f"{W}x{H} -> {cw}x{ch}")


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline,frames", [("restir", 3), ("mcpt", 1), ("reuse", 3), ("gi", 3)])
def test_native_renderer_frames_bit_exact(scene1, scene_dir, oracle_mod, tmp_path, pipeline, frames):
    W, H = 96, 64
    out = str(tmp_path / "img.f32")
    info = json.loads(node("render_frames.js", json.dumps(
        {"sceneDir": scene_dir, "width": W, "height": H, "pipeline": pipeline, "frames": frames, "out": out,
         "present": CANVASES})))
    assert info["frames"] == frames
    img = np.fromfile(out, dtype=np.float32).reshape(H, W, 4)
    fr = oracle_mod.Frame(uniform_for(scene1, W, H, 1), scene1.scene, scene1.geometry, scene1.accel)
    for f in range(1, frames + 1):
        fr.set_frame_index(f)
        if pipeline == "reuse":
            fr.run_reuse_frame()
        elif pipeline == "gi":
            fr.run_gi_frame()
        else:
            fr.run(oracle_mod.PASS_RESTIR if pipeline == "restir" else oracle_mod.PASS_MCPT)
    np.testing.assert_array_equal(np.array(info["uniform"], dtype=np.uint64).astype(np.uint32), fr.uniform)
    np.testing.assert_array_equal(img.view(np.uint32), fr.accum.view(np.uint32))
    for i, (cw, ch, bgra) in enumerate(CANVASES):  # Present: the render pass on the GPU
        got = np.fromfile(f"{out}.present{i}", dtype=np.uint8).reshape(ch, cw, 4)
        np.testing.assert_array_equal(got, oracle_mod.present(fr.accum, cw, ch, bool(bgra)), f"canvas {cw}x{ch}")


# ---------------------------------------------------------------- the reference's World on Node
def _assets_dir(name_or_scene, tmp_path_factory):
    from pathtracerdemo_amd.scene.export import export_meshes
    from pathtracerdemo_amd.scene.world import load_scene_json
    scene = load_scene_json(name_or_scene) if isinstance(name_or_scene, str) else name_or_scene
    d = str(tmp_path_factory.mktemp("assets"))
    with open(os.path.join(d, "scene.json"), "w") as f:
        json.dump(scene, f)
    names = []
    for a in scene["assets"]:
        if a.get("type") == "object" and a.get("meshName") and a["meshName"] not in names:
            names.append(a["meshName"])
    export_meshes(names, os.path.join(d, "meshes"))
    return d, scene


def _py_digest(cs):
    import hashlib
    h = hashlib.sha256()
    for a in (cs.scene, cs.geometry, cs.accel):
        h.update(np.ascontiguousarray(a, dtype="<u4").tobytes())
    return h.hexdigest()


def _odd_scene():
    """DUMMY_SCENE_2 with Euler angles / scales / light vectors that are not f32-exact:
    exercises the quaternion chain (World.ts:14-33), M = S*R*T and M^-1, RectLight's
    normalize(cross) and area, a directional light's normalisation, and the luminance CDF."""
    from pathtracerdemo_amd.scene.world import load_scene_json
    s = load_scene_json("dummy_scene_2")
    for a in s["assets"]:
        if a["type"] == "object":
            a["transform"]["rotation"] = [12.3, 33.3, -7.1]
            a["transform"]["scale"] = [1.1, 0.9, 1.3]
            a["transform"]["position"] = [0.1, -0.2, 0.3]
        elif a["type"] == "directional-light":
            a["lightParams"]["direction"] = [0.3, -1.7, -0.4]
        elif a["type"] == "rect-light":
            a["lightParams"]["u"] = [0.31, 0.02, 0.0]
            a["lightParams"]["v"] = [0.0, 0.05, 0.27]
    return s


@pytest.mark.parametrize("which", ["dummy_scene_1", "c3_interior_32", "odd"])
def test_js_world_serializes_like_the_scene_compiler(which, tmp_path_factory):
    """World.LoadFromScene -> PackWorldData -> Mesh.Serialize -> SerializeWorldData restated in
    JS (pathtracerdemo_amd/js/world.js) gives the Python scene compiler's arrays bit for bit;
    for C1 / C3 that is the golden scene_sha256 the fixtures pin."""
    from pathtracerdemo_amd.scene.world import compile_scene
    scene = _odd_scene() if which == "odd" else which
    d, sc = _assets_dir(scene, tmp_path_factory)
    cs = compile_scene(sc)
    got = json.loads(node("serialize_world.js", d))
    assert got["sha256"] == _py_digest(cs)
    o = cs.offsets
    assert got["offsets"] == [o["mesh_descriptor"], o["material"], o["light"], o["lights_cdf"], o["index"],
                              o["sub_blas_root"], o["blas"]]
    assert (got["instanceCount"], got["lightCount"]) == (cs.instance_count, cs.light_count)
    if which != "odd":
        golden = dict(np.load(os.path.join(ROOT, "tests", "golden",
                                           "c1_24x24_4frames.npz" if which == "dummy_scene_1" else "c3_24x24_2frames.npz")))
        assert bytes.fromhex(got["sha256"]) == golden["scene_sha256"].tobytes()


def test_backend_scene_record_ingests(tmp_path_factory):
    """The backend returns `assets` as a JSON string (SceneResponse.java:24-25); both hosts
    accept that record and compile the same scene as from the parsed array."""
    from pathtracerdemo_amd.scene.world import compile_scene, load_scene_json
    d, sc = _assets_dir("c3_interior_32", tmp_path_factory)
    got = json.loads(node("serialize_world.js", d, "backend"))
    rec = json.dumps({"id": 7, "name": sc["name"], "assets": json.dumps(sc["assets"]), "username": "u"})
    assert got["sha256"] == _py_digest(compile_scene(rec)) == _py_digest(compile_scene("c3_interior_32"))
    with pytest.raises(ValueError):
        compile_scene({"id": 1, "assets": json.dumps({"not": "a list"})})
    assert load_scene_json("c3_interior_32")["assets"] == sc["assets"]


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline,frames", [("reuse", 2), ("restir", 2)])
def test_native_renderer_initialize_from_world_bit_exact(scene3, oracle_mod, tmp_path_factory, pipeline, frames):
    """NativeRenderer.Initialize(World) -- the reference's call, the JS host serializing the
    World itself -- renders C3 frames bit-identical to the oracle."""
    W, H = 80, 48
    d, _ = _assets_dir("c3_interior_32", tmp_path_factory)
    out = str(tmp_path_factory.mktemp("img") / "img.f32")
    info = json.loads(node("render_frames.js", json.dumps(
        {"assetsDir": d, "width": W, "height": H, "pipeline": pipeline, "frames": frames, "out": out})))
    img = np.fromfile(out, dtype=np.float32).reshape(H, W, 4)
    fr = oracle_mod.Frame(uniform_for(scene3, W, H, 1), scene3.scene, scene3.geometry, scene3.accel)
    for f in range(1, frames + 1):
        fr.set_frame_index(f)
        if pipeline == "reuse":
            fr.run_reuse_frame()
        else:
            fr.run(oracle_mod.PASS_RESTIR)
    np.testing.assert_array_equal(np.array(info["uniform"], dtype=np.uint64).astype(np.uint32), fr.uniform)
    np.testing.assert_array_equal(img.view(np.uint32), fr.accum.view(np.uint32))


# ---------------------------------------------------------------- Mesh.Load on Node (GLB + SAH)
@pytest.mark.parametrize("which", ["c3_furnished", "dummy_scene_1"])
def test_js_mesh_load_builds_the_scene_compiler_meshes(which, tmp_path):
    """Mesh.Load on the Node host (js/gltf.js + js/bvh.js: GLB read, node transforms baked in
    three.js's operation order, primitives merged with one group each, SAH BLAS per group) gives
    every mesh the Python scene compiler builds -- positions, normals, uvs, BVH-reordered
    indices, every BLAS root, materials, BVH depth -- bit for bit, and the World serialised from
    those meshes hashes to the scene compiler's arrays (no Python export step)."""
    from pathtracerdemo_amd.scene.world import ASSET_DIR, compile_scene, load_scene_json, mesh_data, serialize_material
    scene = load_scene_json(which)
    sf = tmp_path / "scene.json"
    sf.write_text(json.dumps(scene))
    out = tmp_path / "out"
    out.mkdir()
    got = json.loads(node("load_glb.js", str(sf), ASSET_DIR, str(out)))
    for name in got["names"]:
        md = mesh_data(name)
        rd = lambda ext, dt: np.fromfile(out / f"{name}.{ext}", dtype=dt)  # noqa: E731
        np.testing.assert_array_equal(rd("pos", np.uint32), md.positions.reshape(-1).view(np.uint32), f"{name} positions")
        np.testing.assert_array_equal(rd("nrm", np.uint32), md.normals.reshape(-1).view(np.uint32), f"{name} normals")
        uv = rd("uv", np.uint32)
        np.testing.assert_array_equal(uv, md.uvs.reshape(-1).view(np.uint32) if md.uvs is not None else uv[:0], f"{name} uvs")
        np.testing.assert_array_equal(rd("idx", np.uint32), md.indices, f"{name} indices")
        meta = json.loads((out / f"{name}.json").read_text())
        assert meta["roots"] == len(md.roots) and meta["maxBvhDepth"] == md.max_depth
        for k, r in enumerate(md.roots):
            np.testing.assert_array_equal(rd(f"blas{k}", np.uint32), r, f"{name} BLAS root {k}")
        assert meta["materials"] == [list(serialize_material(m)) for m in md.materials]
    cs = compile_scene(which)
    import hashlib
    h = hashlib.sha256()
    for a in (cs.scene, cs.geometry, cs.accel):
        h.update(np.ascontiguousarray(a, dtype="<u4").tobytes())
    assert got["sha256"] == h.hexdigest()


def test_matrix_nodes_are_decomposed_and_recomposed_like_three():
    """A glTF node `matrix` goes through GLTFLoader's applyMatrix4 -> Matrix4.decompose ->
    compose (never used raw): the Python and JS bakers agree bit for bit on rotated, scaled,
    mirrored (negative determinant) and sheared matrices, and the recomposed matrix equals the
    raw TRS matrix to f64 rounding.  (three.js itself is absent: parity against the library
    is unpinned; this pins the two hosts to one restatement.)"""
    import math
    from pathtracerdemo_amd.scene import gltf as G
    rng = np.random.default_rng(7)
    cases = []
    for k in range(6):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        ang = rng.uniform(-math.pi, math.pi)
        q = [*(ax * math.sin(ang / 2)), math.cos(ang / 2)]
        sc = list(rng.uniform(0.2, 3.0, size=3))
        if k % 2:
            sc[k % 3] = -sc[k % 3]  # mirrored
        cases.append(G._compose(list(rng.normal(size=3) * 4), q, sc))
    cases.append([1.0, 0.0, 0.0, 0.0, 0.5, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 1.0, 2.0, 3.0, 1.0])  # shear
    n_regular = len(cases)
    # zero-scale columns (a collapsed node): JS divides by zero to Infinity / NaN, Python must too
    cases.append([0.0, 0.0, 0.0, 0.0, 0.0, 2.0, 0.0, 0.0, 0.0, 0.0, 3.0, 0.0, 1.0, 2.0, 3.0, 1.0])
    cases.append([0.0] * 12 + [4.0, 5.0, 6.0, 1.0])
    want = [G._node_local_matrix({"matrix": m}) for m in cases]
    for w in want[n_regular:]:
        assert np.isnan(np.array(w, dtype=np.float64)[:12]).any()  # (three.js's result: NaN rotation)
    for m, w in zip(cases[:n_regular - 1], want[:n_regular - 1]):
        np.testing.assert_allclose(w, m, rtol=0, atol=1e-12 * max(1.0, max(abs(v) for v in m)))
    src = ("const G = require('./pathtracerdemo_amd/js/gltf.js');"
           "const ms = JSON.parse(require('fs').readFileSync(0, 'utf8'));"
           "process.stdout.write(JSON.stringify(ms.map((m) => G.localMatrix({ matrix: m }))));")
    p = subprocess.run([NODE, "-e", src], input=json.dumps(cases), capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    assert len(got) == len(want)
    for g, w in zip(got, want):  # (JSON carries -0 as 0 and NaN / Infinity as null: compared as values)
        w = np.array(w, dtype=np.float64)
        w[~np.isfinite(w)] = np.nan
        g = np.array([np.nan if v is None else v for v in g], dtype=np.float64)
        assert np.array_equal(g, w, equal_nan=True)
