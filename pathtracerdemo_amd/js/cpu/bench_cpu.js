'use strict';
/**
 * bench_cpu.js -- the JS CPU baseline of SURVEY.md §8(d): pt_cpu.js's ReSTIR frame (PT_01 ->
 * PT_1 -> PT_4, the reference's live pipeline) on `threads` worker_threads, rows interleaved,
 * timed by wall clock around the render only.
 *
 * usage: node bench_cpu.js <scene_dir> <uniform.u32> <threads> [row_begin row_end] [out_prefix]
 * prints {"seconds", "samples", "threads", "rows", "msamples_per_s"}; with out_prefix also
 * writes <out_prefix>.{gbuffer,reservoir,accum}.bin (full-frame buffers, for the tests).
 */
const fs = require('fs');
const path = require('path');
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');
const { CpuTracer } = require('./pt_cpu');

function sharedU32(src) {
  const sab = new SharedArrayBuffer(src.byteLength);
  new Uint32Array(sab).set(src);
  return sab;
}

if (isMainThread) {
  const [sceneDir, uniformFile, threadsArg, rb, re, outPrefix] = process.argv.slice(2);
  const { loadCompiledScene } = require(path.join(__dirname, '..', 'scene_io'));
  const world = loadCompiledScene(sceneDir);
  const ub = fs.readFileSync(uniformFile);
  const uniform = new Uint32Array(33);
  new Uint8Array(uniform.buffer).set(ub.subarray(0, 132));
  const W = uniform[0], H = uniform[1];
  const y0 = rb === undefined ? 0 : Number(rb), y1 = re === undefined ? H : Number(re);
  const threads = Math.max(1, Number(threadsArg) || require('os').cpus().length);
  const bufs = {
    uniform: sharedU32(uniform), scene: sharedU32(world.scene), geometry: sharedU32(world.geometry),
    accel: sharedU32(world.accel.length ? world.accel : new Uint32Array(1)),
    gb: new SharedArrayBuffer(W * H * 16), res: new SharedArrayBuffer(W * H * 128), accum: new SharedArrayBuffer(W * H * 16),
  };
  let ready = 0, done = 0, t0 = 0;
  const workers = [];
  for (let k = 0; k < threads; ++k) {
    const rows = [];
    for (let y = y0 + k; y < y1; y += threads) rows.push(y);
    const w = new Worker(__filename, { workerData: { ...bufs, rows } });
    w.on('message', (m) => {
      if (m === 'ready' && ++ready === threads) {
        t0 = process.hrtime.bigint();
        for (const x of workers) x.postMessage('go');
      } else if (m === 'done' && ++done === threads) {
        const seconds = Number(process.hrtime.bigint() - t0) / 1e9;
        const samples = W * (y1 - y0);
        if (outPrefix) {
          fs.writeFileSync(outPrefix + '.gbuffer.bin', Buffer.from(bufs.gb));
          fs.writeFileSync(outPrefix + '.reservoir.bin', Buffer.from(bufs.res));
          fs.writeFileSync(outPrefix + '.accum.bin', Buffer.from(bufs.accum));
        }
        process.stdout.write(JSON.stringify({ seconds, samples, threads, rows: [y0, y1],
          msamples_per_s: samples / seconds / 1e6 }) + '\n');
        for (const x of workers) x.terminate();
      }
    });
    w.on('error', (e) => { console.error(e); process.exit(1); });
    workers.push(w);
  }
} else {
  const d = workerData;
  const tracer = new CpuTracer(new Uint32Array(d.uniform), new Uint32Array(d.scene), new Uint32Array(d.geometry),
    new Uint32Array(d.accel));
  const gb = new Uint32Array(d.gb), res = new Uint32Array(d.res), accum = new Float32Array(d.accum);
  parentPort.on('message', () => {
    tracer.frameRows(d.rows, gb, res, accum);
    parentPort.postMessage('done');
  });
  parentPort.postMessage('ready');
}
