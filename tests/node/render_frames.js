'use strict';
// Renders `frames` frames through NativeRenderer (Update + RenderAsync, as WebGPUEngine's
// loop does) and writes the accumulated RGBA f32 image to `out`.  argv: JSON request.
const fs = require('fs');
const { NativeRenderer } = require('../../pathtracerdemo_amd/js/NativeRenderer');
const { loadCompiledScene } = require('../../pathtracerdemo_amd/js/scene_io');

async function main() {
  const req = JSON.parse(process.argv[2]);
  const r = new NativeRenderer(req.width, req.height, { pipeline: req.pipeline, device: 0 });
  await r.Initialize(loadCompiledScene(req.sceneDir));
  for (let f = 0; f < req.frames; f++) {
    r.Update();
    await r.RenderAsync();
  }
  const img = r.ReadImage();
  fs.writeFileSync(req.out, Buffer.from(img.buffer, img.byteOffset, img.byteLength));
  const st = r.GetStats();
  r.Destroy();
  process.stdout.write(JSON.stringify({ frames: st.frames, uniform: Array.from(r.Uniform) }));
}
main().catch((e) => { console.error(e.stack || String(e)); process.exit(1); });
