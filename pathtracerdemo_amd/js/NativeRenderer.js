'use strict';
/**
 * NativeRenderer -- the drop-in for the reference's Renderer_TEST
 * (apps/frontend/src/graphics-core/Renderer_TEST.ts) over the ptx_node N-API addon.
 *
 * Same surface: constructor, async Initialize(world), Update(), Render(), GetCamera(),
 * ResetFrameCount(); WebGPUEngine's loop (GC/service/WebGPUEngine.ts:199-200) calls
 * Update() then Render() per tick exactly as before, and nothing else.  Like Renderer_TEST.Render
 * (Renderer_TEST.ts:233-258, which ends by drawing into the canvas it was constructed with),
 * Render() paints the canvas it was given: when the canvas offers getContext('2d'), the reference's
 * render pass (the fullscreen quad + FragmentShader.wgsl's fixed 600 x 450 texel window, unorm8)
 * runs on the GPU behind the frame (ptx_present_async) and its bytes go to putImageData once they
 * have landed -- polled off the event loop, never waited for; while one present is in flight a
 * newer frame is presented after it, so the canvas always ends on the newest finished frame
 * (PresentedSerial: the Render() call it shows; PresentIdle(): a promise for "nothing in flight").
 * ReadImage / RenderAsync(out) give the accumulated RGBA f32 image; Present(canvasW, canvasH)
 * is the same render pass, blocking, into RGBA (putImageData) or BGRA (a bgra8unorm WebGPU
 * canvas) bytes.  presentImage does it on the host for a frame gathered from row bands
 * (renderBands).
 *
 * `world` is the reference's own World (./world.js: World.LoadFromScene over the Scene JSON,
 * meshes in ResourceManager.MeshPool), serialized here by SerializeWorldData exactly as
 * Renderer_TEST.CreateGPUResources does (Renderer_TEST.ts:445-460) -- or, equivalently, an
 * already serialized { scene, geometry, accel: Uint32Array, offsets: number[7],
 * instanceCount, lightCount } (scene_io.loadCompiledScene reads one from disk).
 * There is no CPU fallback: a missing addon or libptx.so throws at require time.
 */
const path = require('path');
const { Camera } = require('./Camera');
const { mat4 } = require('./wgpu_math');
const { SerializeWorldData } = require('./world');

const addon = require(path.join(__dirname, '..', 'ptx_node.node'));

const PIPELINE = { restir: 0, mcpt: 1, reuse: 2, gi: 3 };
const PASS = { GBUFFER: 0, INIT: 1, FINAL: 2, MCPT: 3, TRACE: 4, WAVE_TRACE: 5, WAVE_LOGIC: 6, FRAME: 7,
  TEMPORAL: 8, SPATIAL: 9, PASS_GROUP: 10 };
const BUF = { GBUFFER: 0, RESERVOIR: 1, ACCUM: 2, COUNTERS: 3, RESERVOIR_HIST: 4 };
const FLAGS = { COUNT_WORK: 1, SIMPLE_KERNELS: 2, TIME_LAUNCHES: 16 };
const UNIFORM_WORDS = 33;

/** The 33-word uniform block of Renderer_TEST.Update (Renderer_TEST.ts:165-206). */
function buildUniform(width, height, camera, frameCount, world) {
  const data = new ArrayBuffer(4 * UNIFORM_WORDS);
  const f32 = new Float32Array(data);
  const u32 = new Uint32Array(data);
  const loc = camera.GetLocation();
  const vpInv = mat4.invert(camera.GetViewProjectionMatrix());
  u32[0] = width;
  u32[1] = height;
  u32[2] = 10; // Max Bounce (unused by the kernels)
  u32[3] = 1;  // SPP
  for (let i = 0; i < 16; i++) f32[4 + i] = vpInv[i];
  f32[20] = loc[0];
  f32[21] = loc[1];
  f32[22] = loc[2];
  u32[23] = frameCount;
  for (let i = 0; i < 7; i++) u32[24 + i] = world.offsets[i];
  u32[31] = world.instanceCount;
  u32[32] = world.lightCount;
  return u32;
}

function isCanvas(x) {
  return !!x && typeof x === 'object' && typeof x.width === 'number' && typeof x.height === 'number';
}

// the next turn of the event loop (Node: setImmediate; a browser: a zero timeout)
const soon = typeof setImmediate === 'function' ? setImmediate : (fn) => setTimeout(fn, 0);

class NativeRenderer {
  /**
   * Three call forms:
   *   new NativeRenderer(adapter, device, canvas, [options])  -- Renderer_TEST's own
   *     (Renderer_TEST.ts:83-88, WebGPUEngine.ts:83); adapter / device are not used;
   *   new NativeRenderer(canvas, [options]);
   *   new NativeRenderer(width, height, [options]).
   * `canvas` is anything with numeric width / height (an HTMLCanvasElement, an OffscreenCanvas,
   * a plain object): like Renderer_TEST, Initialize() reads its size each time it is called, so
   * WebGPUEngine.resize (set canvas.width / height, then Initialize(world), WebGPUEngine.ts:132-142)
   * recreates the handle at the new size.
   * @param {object} [options] {pipeline: 'restir'|'mcpt'|'reuse'|'gi', device, rowBegin, rowEnd, flags,
   *   reuseRadius, reuseNeighbors, temporalCap}
   */
  constructor(a, b, c, d) {
    let options;
    if (typeof a === 'number') {
      this.Canvas = null;
      this.Width = a;
      this.Height = b;
      options = c || {};
    } else if (isCanvas(a)) {
      this.Canvas = a;
      options = b || {};
    } else if (isCanvas(c)) {
      this.Canvas = c;
      options = d || {};
    } else {
      throw new TypeError('NativeRenderer: expected (width, height), (canvas) or (adapter, device, canvas)');
    }
    if (this.Canvas) {
      this.Width = this.Canvas.width;
      this.Height = this.Canvas.height;
    }
    this.Options = options;
    this.Pipeline = options.pipeline || 'restir';
    if (!(this.Pipeline in PIPELINE)) throw new Error(`unknown pipeline ${this.Pipeline}`);
    this.Handle = null;
    this.createHandle();
    this.World = null;
    this.Camera = null;
    this.FrameCount = 0;
    this.Uniform = null;
    // canvas painting (Render): the 2D context, the present in flight, its waiters
    this.Context2D = undefined;
    this.RenderSerial = 0;
    this.PresentedSerial = 0;
    this.PresentInFlight = null;
    this.PresentWanted = false;
    this.PresentWaiters = [];
    this.PresentError = null;
  }

  /** A handle for this.Width x this.Height (rows rowBegin..rowEnd of it). */
  createHandle() {
    const o = this.Options;
    this.RowBegin = o.rowBegin || 0;
    this.RowEnd = o.rowEnd || this.Height;
    this.Handle = addon.create({
      width: this.Width, height: this.Height, rowBegin: this.RowBegin, rowEnd: this.RowEnd,
      device: o.device === undefined ? -1 : o.device,
      pipeline: PIPELINE[this.Pipeline], flags: o.flags || 0,
      reuseRadius: o.reuseRadius || 0, reuseNeighbors: o.reuseNeighbors || 0,
      temporalCap: o.temporalCap || 0,
    });
  }

  GetCamera() { return this.Camera; }

  ResetFrameCount() { this.FrameCount = 0; }

  /**
   * Renderer_TEST.Initialize (:141-163): the canvas's current size (a changed size recreates the
   * handle, as DestroyGPUResources + CreateGPUResources do), a new camera at (0,0,6) with
   * yaw / pitch 0, FrameCount 0, the world uploaded.
   */
  async Initialize(world) {
    // a reference World is serialized here (SerializeWorldData); a serialized one is taken as is
    if (world && world.InstancesPool instanceof Map) world = SerializeWorldData(world);
    if (!world || !(world.scene instanceof Uint32Array) || !Array.isArray(world.offsets) || world.offsets.length !== 7) {
      throw new TypeError('Initialize: expected a World or a serialized world {scene, geometry, accel, offsets[7]}');
    }
    if (this.Canvas && (this.Canvas.width !== this.Width || this.Canvas.height !== this.Height)) {
      if (this.Options.rowBegin || this.Options.rowEnd) {
        throw new Error('Initialize: a row-band renderer cannot follow a canvas resize');
      }
      if (!(this.Canvas.width > 0 && this.Canvas.height > 0)) throw new RangeError('Initialize: empty canvas');
      this.dropPresent();
      if (this.Handle) addon.destroy(this.Handle);
      this.Handle = null;
      this.Width = this.Canvas.width;
      this.Height = this.Canvas.height;
      this.createHandle();
    }
    this.Camera = new Camera(this.Width, this.Height);
    this.Camera.SetLocationFromXYZ(0, 0, 6);
    this.Camera.SetYaw(0);
    this.Camera.SetPitch(0);
    this.World = world;
    this.ResetFrameCount();
    addon.uploadScene(this.Handle, world.scene, world.geometry, world.accel);
    addon.resetAccumulation(this.Handle);
  }

  /** Renderer_TEST.Update (:165-206): FrameCount++, then the uniform block. */
  Update() {
    this.FrameCount++;
    this.Uniform = buildUniform(this.Width, this.Height, this.Camera, this.FrameCount, this.World);
    addon.setFrame(this.Handle, this.Uniform);
  }

  /**
   * Renderer_TEST.Render (:208-261): all passes + accumulation, asynchronous on the GPU, then the
   * render pass into the canvas (:233-258) when it has a 2D context -- enqueued behind the frame,
   * painted when its bytes land (the event loop is never blocked).
   */
  Render() {
    addon.render(this.Handle);
    this.RenderSerial++;
    if (this.context2D()) {
      if (this.PresentInFlight) this.PresentWanted = true;
      else this.startPresent();
    }
  }

  /** The canvas's 2D context (looked up once; null when the canvas has none, e.g. in a worker). */
  context2D() {
    if (this.Context2D === undefined) {
      const c = this.Canvas;
      this.Context2D = (c && typeof c.getContext === 'function' && c.getContext('2d')) || null;
    }
    return this.Context2D;
  }

  startPresent() {
    const ctx = this.context2D();
    const w = this.Canvas.width, h = this.Canvas.height;
    this.PresentWanted = false;
    if (!(w > 0 && h > 0)) return;  // (nothing to paint on an empty canvas)
    let image;
    try {
      image = ctx.createImageData(w, h);
      addon.presentAsync(this.Handle, w, h, false);
    } catch (e) {  // painting never breaks the render loop: the error is kept for the host to read
      this.PresentError = e;
      return;
    }
    this.PresentInFlight = { serial: this.RenderSerial, image, handle: this.Handle };
    soon(() => this.pollPresent(0));
  }

  pollPresent(tries) {
    const f = this.PresentInFlight;
    if (!f || f.handle !== this.Handle) return;  // dropped (Destroy, a resize)
    let done;
    try {
      done = addon.presentPoll(this.Handle, f.image.data);
    } catch (e) {
      if (/in flight on this handle/.test(String(e && e.message))) {  // a RenderAsync owns the handle
        setTimeout(() => this.pollPresent(tries + 1), 1);
        return;
      }
      this.PresentInFlight = null;
      this.PresentError = e;
      this.settlePresent();
      return;
    }
    if (!done) {  // the first few polls on the next turns, then every millisecond
      if (tries < 8) soon(() => this.pollPresent(tries + 1));
      else setTimeout(() => this.pollPresent(tries + 1), 1);
      return;
    }
    this.PresentInFlight = null;
    this.PresentedSerial = f.serial;
    this.context2D().putImageData(f.image, 0, 0);
    if (this.PresentWanted) this.startPresent();
    else this.settlePresent();
  }

  settlePresent() {
    const ws = this.PresentWaiters;
    this.PresentWaiters = [];
    for (const r of ws) r();
  }

  /** Resolves once no present is in flight (the canvas shows the newest rendered frame). */
  PresentIdle() {
    if (!this.PresentInFlight) return Promise.resolve(this.PresentedSerial);
    return new Promise((resolve) => this.PresentWaiters.push(() => resolve(this.PresentedSerial)));
  }

  dropPresent() {
    this.PresentInFlight = null;
    this.PresentWanted = false;
    this.settlePresent();
  }

  /** Render off the event loop; resolves once the frame (and the optional copy) is done. */
  RenderAsync(out) { return addon.renderAsync(this.Handle, out || null); }

  /** The accumulated band image, RGBA f32 (the reference's Scene texture). */
  ReadImage(out) {
    const img = out || new Float32Array((this.RowEnd - this.RowBegin) * this.Width * 4);
    addon.readBuffer(this.Handle, BUF.ACCUM, img);
    return img;
  }

  /**
   * Renderer_TEST.Render's render pass (Renderer_TEST.ts:233-255) onto a canvasW x canvasH canvas
   * (default: the image size): Uint8ClampedArray of canvasW * canvasH * 4 bytes, RGBA (bgra false:
   * ImageData for putImageData) or BGRA (bgra true); row 0 = the canvas's top row.
   */
  Present(canvasW = this.Width, canvasH = this.Height, bgra = false, out = null) {
    const px = out || new Uint8ClampedArray(canvasW * canvasH * 4);
    addon.present(this.Handle, canvasW, canvasH, bgra, px);
    return px;
  }

  RunPass(pass) { addon.runPass(this.Handle, pass); }
  Synchronize() { addon.synchronize(this.Handle); }
  GetStats() { return addon.getStats(this.Handle); }
  Trace(rays, hits, epsMode = 1) { addon.trace(this.Handle, rays, hits, epsMode); }

  /** DestroyGPUResources (:462-476). */
  Destroy() {
    this.dropPresent();
    if (this.Handle) addon.destroy(this.Handle);
    this.Handle = null;
  }
}

/**
 * The same render pass on the host, for a frame gathered from row bands (Renderer.renderBands'
 * image, rows 0 .. height): canvas pixel (x, y) shows texel (floor((2x+1)*600 / 2canvasW),
 * floor((2canvasH-2y-1)*450 / 2canvasH)) -- FragmentShader.wgsl:7-10's PixelUV * (600, 450) of the
 * quad's VertexShader.wgsl UV at the pixel centre, in exact integers -- clamped to [0, 1] and
 * rounded half to even to unorm8 (ptx_present's rules; out-of-bounds texels read 0).
 */
function presentImage(img, width, height, canvasW, canvasH, bgra = false, out = null) {
  const px = out || new Uint8ClampedArray(canvasW * canvasH * 4);
  const f = new Float32Array(1);
  const unorm8 = (x) => {
    if (!(x > 0)) return 0; // (NaN, <= 0)
    if (x >= 1) return 255;
    f[0] = Math.fround(x * 255); // the f32 product, then round half to even
    const v = f[0], fl = Math.floor(v), d = v - fl;
    return d > 0.5 || (d === 0.5 && (fl % 2) === 1) ? fl + 1 : fl;
  };
  for (let y = 0; y < canvasH; y++) {
    const ty = Math.floor(((2 * canvasH - 2 * y - 1) * 450) / (2 * canvasH));
    for (let x = 0; x < canvasW; x++) {
      const tx = Math.floor(((2 * x + 1) * 600) / (2 * canvasW));
      const o = 4 * (y * canvasW + x);
      let r = 0, g = 0, b = 0;
      if (tx < width && ty < height) {
        const i = 4 * (ty * width + tx);
        r = unorm8(img[i]); g = unorm8(img[i + 1]); b = unorm8(img[i + 2]);
      }
      px[o] = bgra ? b : r; px[o + 1] = g; px[o + 2] = bgra ? r : b; px[o + 3] = 255;
    }
  }
  return px;
}

module.exports = { NativeRenderer, buildUniform, presentImage, addon, PASS, BUF, FLAGS, UNIFORM_WORDS };
