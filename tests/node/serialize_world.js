'use strict';
// World.LoadFromScene + SerializeWorldData on the Node host (pathtracerdemo_amd/js/world.js):
// argv[2] = an export.export_scene_assets directory (scene.json + meshes/), argv[3] = 'backend'
// to feed the scene as the backend's record (assets as a JSON string).  Prints the sha256 of
// the three arrays (as tests/golden/make_golden.py's scene_digest) and the uniform's words.
const fs = require('fs');
const crypto = require('crypto');
const W = require('../../pathtracerdemo_amd/js/world');

const dir = process.argv[2];
let rec = JSON.parse(fs.readFileSync(dir + '/scene.json', 'utf8'));
if (process.argv[3] === 'backend') rec = JSON.stringify({ ...rec, id: 7, assets: JSON.stringify(rec.assets) });
const scene = W.sceneFromBackend(rec);
W.ResourceManager.LoadCompiledAssets(dir + '/meshes', W.sceneMeshNames(scene));
const world = new W.World();
world.LoadFromScene(scene);
const s = W.SerializeWorldData(world);
const h = crypto.createHash('sha256');
for (const a of [s.scene, s.geometry, s.accel]) h.update(Buffer.from(a.buffer, a.byteOffset, a.byteLength));
process.stdout.write(JSON.stringify({ sha256: h.digest('hex'), offsets: Array.from(s.offsets),
  instanceCount: s.instanceCount, lightCount: s.lightCount, maxBvhDepth: s.maxBvhDepth,
  sizes: [s.scene.length, s.geometry.length, s.accel.length] }));
