'use strict';
/**
 * Reads a compiled scene directory (pathtracerdemo_amd/scene/export.py) into the shape
 * NativeRenderer.Initialize takes: the three u32 arrays of Renderer_TEST.SerializeWorldData
 * (GC/Renderer_TEST.ts:267-420) plus Offsets[] and the instance / light counts.
 */
const fs = require('fs');
const path = require('path');

function readU32(file) {
  const buf = fs.readFileSync(file);
  if (buf.byteLength % 4) throw new Error(`${file}: size ${buf.byteLength} is not a multiple of 4`);
  // copy into an aligned buffer (Buffer pooling may leave byteOffset unaligned)
  const out = new Uint32Array(buf.byteLength / 4);
  new Uint8Array(out.buffer).set(buf);
  return out;
}

function loadCompiledScene(dir) {
  const meta = JSON.parse(fs.readFileSync(path.join(dir, 'world.json'), 'utf8'));
  if (!Array.isArray(meta.offsets) || meta.offsets.length !== 7) throw new Error(`${dir}: world.json needs 7 offsets`);
  return {
    name: meta.name,
    scene: readU32(path.join(dir, 'scene.u32')),
    geometry: readU32(path.join(dir, 'geometry.u32')),
    accel: readU32(path.join(dir, 'accel.u32')),
    offsets: meta.offsets,
    instanceCount: meta.instanceCount,
    lightCount: meta.lightCount,
    triangleCount: meta.triangleCount,
    maxBvhDepth: meta.maxBvhDepth,
  };
}

module.exports = { loadCompiledScene };
