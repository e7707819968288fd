'use strict';
// NativeRenderer.Render's canvas painting with a stand-in addon (no GPU): the addon's
// presentAsync / presentPoll pair is simulated -- a present "lands" a random 0-3 event-loop turns
// after it was enqueued and carries the frame it followed -- so the JS scheduling is checked on the
// CPU: Render() never waits, every putImageData shows the frame of the Render() call it names
// (PresentedSerial), puts come in frame order, the canvas ends on the newest frame, and a resize
// (Initialize on a new canvas size) drops the present in flight.
const path = require('path');
const addonPath = path.join(__dirname, '..', '..', 'pathtracerdemo_amd', 'ptx_node.node');
let seq = 0;
let now = 0;                                     // event-loop turns elapsed
const rnd = (() => { let s = 12345; return () => { s = (s * 1103515245 + 12345) >>> 0; return s / 4294967296; }; })();
const fake = {
  create(cfg) { return { id: ++seq, w: cfg.width, h: cfg.height, frames: 0, pending: null, destroyed: false }; },
  uploadScene() {}, resetAccumulation() {}, setFrame() {},
  render(h) { h.frames++; },
  presentAsync(h, w, hh, bgra) {
    if (h.pending) throw new Error('ptx_present_async: a present is in flight');
    h.pending = { frame: h.frames, w, hh, readyAt: now + Math.floor(rnd() * 4) };
  },
  presentPoll(h, out) {
    if (!h.pending) throw new Error('ptx_present_poll: no present in flight');
    if (now < h.pending.readyAt) return false;
    out.fill(h.pending.frame & 255);
    h.pending = null;
    return true;
  },
  destroy(h) { h.destroyed = true; },
};
require.cache[addonPath] = { id: addonPath, filename: addonPath, loaded: true, exports: fake };
const { NativeRenderer } = require('../../pathtracerdemo_amd/js/NativeRenderer');
const tick = () => new Promise((r) => setImmediate(() => { now++; r(); }));

async function main() {
  const puts = [];
  const canvas = { width: 8, height: 6 };
  const ctx = {
    createImageData: (w, h) => ({ width: w, height: h, data: new Uint8ClampedArray(w * h * 4) }),
    putImageData: (img) => puts.push({ serial: r.PresentedSerial, w: img.width, h: img.height, v: img.data[0],
      uniform: img.data.every((x) => x === img.data[0]) }),
  };
  canvas.getContext = (k) => (k === '2d' ? ctx : null);
  const r = new NativeRenderer(null, null, canvas, {});
  const world = { scene: new Uint32Array(4), geometry: new Uint32Array(4), accel: new Uint32Array(4),
    offsets: [0, 0, 0, 0, 0, 0, 0], instanceCount: 0, lightCount: 0 };
  await r.Initialize(world);
  const frameOf = {};                            // serial -> frame number on its handle
  let resizedAt = -1;
  for (let t = 0; t < 40; t++) {
    if (t === 25) {                              // a resize: a new handle, the present in flight dropped
      canvas.width = 5; canvas.height = 4;
      await r.Initialize(world);
      resizedAt = r.RenderSerial;
    }
    r.Update();
    const t0 = Date.now();
    r.Render();
    if (Date.now() - t0 > 50) throw new Error('Render waited');
    frameOf[r.RenderSerial] = r.Handle.frames;
    if (rnd() < 0.5) await tick();               // some ticks yield, some do not (bursts of frames)
  }
  for (let k = 0; k < 20; k++) await tick();
  await r.PresentIdle();
  process.stdout.write(JSON.stringify({ puts, frameOf, resizedAt, last: r.RenderSerial }));
}
main().catch((e) => { console.error(e.stack || String(e)); process.exit(1); });
