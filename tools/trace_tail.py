"""Launch tails of trace_queue's dynamic batches, from the diagnostic build's per-batch records.

usage (GPU box):  make -C pathtracerdemo_amd/csrc wgt
                  PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so python tools/trace_tail.py [--out f.json]

Renders the headline configuration the way bench.py's launch-timed region does (one launch
sequence, one frame in flight, dynamic trace batches) and, per trace launch of the measured
frames, reports: the span (first wave start -> last wave end), the drain point (the first wave
to exit: waves exit only once every batch head is empty), the tail after it and the mean
resident waves, plus the batch-duration spread.  Then two what-ifs on the measured batch
durations, by greedy list scheduling on the launch's plateau wave count: the batches in their
measured dequeue order, and longest-first -- either with the true durations (a bound) or keyed
by the SAME batch index's duration in the previous frame (what a scheduler could know).
"""
import argparse
import ctypes
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KID_TRACE, KID_BATCH, KID_BATCH_DBG = 1, 12, 15


def list_schedule(durs, slots):
    """Makespan of running `durs` in order on `slots` identical workers (each takes the next job
    when it frees)."""
    if len(durs) == 0:
        return 0.0
    h = [0.0] * int(slots)
    heapq.heapify(h)
    for d in durs:
        heapq.heappush(h, heapq.heappop(h) + d)
    return max(h)


def launches(rec):
    """Split one frame's records into trace launches (single stream: launches do not overlap)."""
    kid = (rec[:, 2] >> np.uint64(32)).astype(np.int64) & 0x7F
    tw = rec[kid == KID_TRACE]
    ib = np.nonzero(kid == KID_BATCH)[0]
    ib = ib[ib + 1 < len(rec)]
    ib = ib[kid[ib + 1] == KID_BATCH_DBG]
    # a batch record + its work breakdown as one 8-word row
    tb = np.concatenate([rec[ib], rec[ib + 1]], axis=1)
    order = np.argsort(tw[:, 0])
    tw = tw[order]
    out, cur, end = [], [], -1
    for r in tw:
        if cur and int(r[0]) > end:
            out.append(np.array(cur))
            cur = []
        cur.append(r)
        end = max(end, int(r[1]))
    if cur:
        out.append(np.array(cur))
    res = []
    for w in out:
        t0, t1 = int(w[:, 0].min()), int(w[:, 1].max())
        b = tb[(tb[:, 0] >= t0) & (tb[:, 1] <= t1)]
        res.append((w, b))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--pipeline", default="reuse")
    ap.add_argument("--scene", default="c3_interior_32")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    assert "WGT" in os.environ.get("PTX_AB", "") and "wgt" in os.environ.get("PTX_LIB_PATH", ""), \
        "run with PTX_AB=WGT PTX_LIB_PATH=<libptx_wgt.so>"
    from pathtracerdemo_amd import _native as N
    from pathtracerdemo_amd.renderer import Renderer
    from pathtracerdemo_amd.scene.world import compile_scene
    lib = N.load()
    lib.ptx_diag_wave_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.ptx_diag_wave_times.restype = ctypes.c_int
    r = Renderer(a.width, a.height, device=0, pipeline=a.pipeline, single_stream=True, time_launches=True)
    r.Initialize(compile_scene(a.scene))
    for _ in range(3):
        r.Update()
        r.Render()
    buf = np.zeros((1 << 20, 4), dtype=np.uint64)
    r.synchronize()
    lib.ptx_diag_wave_times(r._h, buf.ctypes.data, 1 << 20)  # drop the warm-up records
    frames = []
    for _ in range(a.frames):
        r.Update()
        r.Render()
        r.synchronize()
        n = lib.ptx_diag_wave_times(r._h, buf.ctypes.data, 1 << 20)
        frames.append(launches(buf[:n].copy()))
    r.close()
    summary = []
    nbhd = {}
    print(f"{a.pipeline} {a.scene} {a.width}x{a.height}: {len(frames[0])} trace launches per frame")
    print("launch  span_us  drain_us  tail_us  tail%  waves  mean_res  plateau  batches  b_p50  b_p99  b_max"
          "  sched_meas  lpt_true  lpt_prev  corr_prev")
    for fi, fr in enumerate(frames):
        for li, (w, b) in enumerate(fr):
            t0 = w[:, 0].min()
            ws = (w[:, 0] - t0) / 100.0
            we = (w[:, 1] - t0) / 100.0
            span = we.max()
            drain = we.min()
            tail = span - drain
            mean_res = (we - ws).sum() / span
            # plateau: resident waves at the drain point (every slot still busy)
            plateau = int(((ws <= drain) & (we >= drain)).sum())
            bs = (b[:, 0] - t0) / 100.0
            bd = (b[:, 1] - b[:, 0]) / 100.0
            bi = (b[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
            meas = list_schedule(bd[np.argsort(bs)], plateau)
            lpt_true = list_schedule(np.sort(bd)[::-1], plateau)
            lpt_prev = corr = None
            if fi > 0 and li < len(frames[fi - 1]):
                pb = frames[fi - 1][li][1]
                pbi = (pb[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
                pd = np.zeros(max(int(pbi.max()) + 1, int(bi.max()) + 1) if len(pbi) else int(bi.max()) + 1)
                pd[pbi] = (pb[:, 1] - pb[:, 0]) / 100.0
                key = pd[bi] if len(pd) > bi.max() else np.zeros_like(bd)
                lpt_prev = list_schedule(bd[np.argsort(-key, kind="stable")], plateau)
                corr = float(np.corrcoef(key, bd)[0, 1]) if len(bd) > 2 else None
                # the previous frame's durations around the same batch index (neighbouring tiles):
                # max over a +-W window -- a per-region cost a scheduler could know
                for W in (4, 16, 64):
                    if len(pd):
                        pm = np.maximum.reduce([np.roll(np.pad(pd, W), -s)[W:W + len(pd)] for s in range(-W, W + 1)])
                        nk = pm[np.minimum(bi, len(pm) - 1)]
                        row_nb = list_schedule(bd[np.argsort(-nk, kind="stable")], plateau)
                        nbhd[W] = nbhd.get(W, []) + [(meas, row_nb, lpt_true)]
            row = {"frame": fi, "launch": li, "span_us": span, "drain_us": drain, "tail_us": tail,
                   "waves": int(len(w)), "mean_resident": mean_res, "plateau": plateau, "batches": int(len(b)),
                   "batch_p50": float(np.percentile(bd, 50)) if len(bd) else 0.0,
                   "batch_p99": float(np.percentile(bd, 99)) if len(bd) else 0.0,
                   "batch_max": float(bd.max()) if len(bd) else 0.0,
                   "sched_measured_order_us": meas, "lpt_true_us": lpt_true, "lpt_prev_frame_us": lpt_prev,
                   "corr_prev_frame": corr}
            summary.append(row)
            print(f"{fi}.{li:<4d} {span:8.1f} {drain:9.1f} {tail:8.1f} {100*tail/span:5.1f} {len(w):6d} {mean_res:9.0f}"
                  f" {plateau:8d} {len(b):8d} {row['batch_p50']:6.1f} {row['batch_p99']:6.1f} {row['batch_max']:6.1f}"
                  f" {meas:11.1f} {lpt_true:9.1f} " + (f"{lpt_prev:9.1f} {corr:10.3f}" if lpt_prev is not None else ""))
    for W, v in sorted(nbhd.items()):
        m, nb, lt = (sum(x[i] for x in v) for i in range(3))
        print(f"longest-first by the previous frame's max over batches +-{W}: summed makespan {nb:9.1f} us "
              f"(measured order {m:9.1f}, true longest-first {lt:9.1f})")
    # what the slow batches do: wave-level iterations per region vs duration (last frame)
    allb = np.concatenate([b for _, b in frames[-1]])
    dur = (allb[:, 1] - allb[:, 0]) / 100.0
    refill = (allb[:, 4] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    node = (allb[:, 4] >> np.uint64(32)).astype(np.int64)
    leafp = (allb[:, 5] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    chunks = (allb[:, 5] >> np.uint64(32)).astype(np.int64)
    calls = (allb[:, 6] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    maxslab = allb[:, 7].astype(np.int64)
    order = np.argsort(dur)
    print("\nbatches by duration (last frame): us, refill it, node-loop it, leaf phases, tri chunks, calls, max slab tests/lane")
    for q in (0.5, 0.9, 0.99, 0.999):
        k = order[int(q * (len(order) - 1))]
        print(f"  p{q*100:5.1f}: {dur[k]:7.1f}  {refill[k]:5d} {node[k]:6d} {leafp[k]:5d} {chunks[k]:5d} {calls[k]:3d} {maxslab[k]:6d}")
    print("  slowest 15:")
    for k in order[::-1][:15]:
        print(f"          {dur[k]:7.1f}  {refill[k]:5d} {node[k]:6d} {leafp[k]:5d} {chunks[k]:5d} {calls[k]:3d} {maxslab[k]:6d}")
    for c in sorted(set(calls.tolist())):
        m = calls == c
        print(f"  calls {c}: {m.sum():6d} batches, mean {dur[m].mean():6.1f} us, p99 {np.percentile(dur[m], 99):6.1f} us, "
              f"node-loop it mean {node[m].mean():6.1f}, share of batch time {dur[m].sum() / dur.sum():.3f}")
    if a.out:
        np.savez(a.out.replace(".json", "_batches.npz"), dur=dur, refill=refill, node=node, leaf=leafp, chunks=chunks,
                 calls=calls, maxslab=maxslab)
    for name, v in (("node-loop it", node), ("refill it", refill), ("leaf phases", leafp), ("tri chunks", chunks),
                    ("calls", calls), ("max slab", maxslab)):
        print(f"  corr(duration, {name}) = {np.corrcoef(dur, v)[0, 1]:.3f}; mean {v.mean():.1f}")
    if a.out:
        json.dump(summary, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
