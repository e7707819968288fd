'use strict';
// Mesh.Load on the Node host (pathtracerdemo_amd/js/{gltf,bvh,world}.js): argv[2] = a Scene JSON
// file, argv[3] = the directory of its <mesh>.glb assets, argv[4] = an output directory.  Loads
// every mesh the scene names through ResourceManager.LoadAssets (GLB -> baked, merged geometry ->
// SAH BLAS), writes each mesh's arrays to <out>/<mesh>.{pos,nrm,uv,idx,blas<k>} + <mesh>.json, then
// World.LoadFromScene + SerializeWorldData and prints the sha256 of the three arrays.
const fs = require('fs');
const path = require('path');
const crypto = require('crypto');
const W = require('../../pathtracerdemo_amd/js/world');

(async () => {
  const [sceneFile, assetDir, out] = process.argv.slice(2);
  const scene = W.sceneFromBackend(fs.readFileSync(sceneFile, 'utf8'));
  const names = W.sceneMeshNames(scene);
  const t0 = Date.now();
  await W.ResourceManager.LoadAssets(names, assetDir);
  const loadMs = Date.now() - t0;
  const dump = (file, a) => fs.writeFileSync(path.join(out, file), Buffer.from(a.buffer, a.byteOffset, a.byteLength));
  for (const name of names) {
    const m = W.ResourceManager.MeshPool.get(name);
    dump(`${name}.pos`, m.VertexPositions);
    dump(`${name}.nrm`, m.VertexNormals);
    dump(`${name}.uv`, m.VertexUVs);
    dump(`${name}.idx`, m.IndexArray);
    m.BlasTree.forEach((r, k) => dump(`${name}.blas${k}`, r));
    fs.writeFileSync(path.join(out, `${name}.json`), JSON.stringify({ roots: m.BlasTree.length, maxBvhDepth: m.MaxBvhDepth,
      materials: m.Materials.map((x) => Array.from(x.Serialize())) }));
  }
  const world = new W.World();
  world.LoadFromScene(scene);
  const s = W.SerializeWorldData(world);
  const h = crypto.createHash('sha256');
  for (const a of [s.scene, s.geometry, s.accel]) h.update(Buffer.from(a.buffer, a.byteOffset, a.byteLength));
  process.stdout.write(JSON.stringify({ sha256: h.digest('hex'), names, loadMs }));
})().catch((e) => { console.error(e.stack || String(e)); process.exit(1); });
