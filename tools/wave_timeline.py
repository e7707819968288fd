"""Wave occupancy of one reuse frame, from the diagnostic build's per-wave timing records.

usage (GPU box):  make -C pathtracerdemo_amd/csrc wgt
                  PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so python tools/wave_timeline.py [--out f.json]
Every instrumented kernel's waves log {start, end} on the 100 MHz real-time clock
(PTX_WAVE_TIMER, ptx_device.h).  Prints, over the frame: the resident-wave count per
kernel kind in 20 us bins (the chip holds 256 CUs x 4 SIMDs x the kernel's waves/SIMD), the
time-averaged occupancy, and per kernel the wave-duration spread (what a launch's tail is)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KIDS = {1: "trace", 2: "gbuffer", 3: "init_start", 4: "init_step", 5: "final_start", 6: "final_step",
        7: "temporal_start", 8: "temporal_combine", 9: "spatial_start", 10: "job_step", 11: "spatial_combine"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--pipeline", default="reuse")
    ap.add_argument("--scene", default="c3_interior_32")
    ap.add_argument("--out", default=None)
    ap.add_argument("--bin-us", type=float, default=20.0)
    ap.add_argument("--frames", type=int, default=1, help="frames in the measured window (pipelined frames overlap)")
    ap.add_argument("--single-stream", action="store_true",
                    help="one launch sequence, one frame in flight (PTX_FLAG_SINGLE_STREAM): the launch-timed "
                         "region of bench.py; prints each trace launch's fill (wave-us over span x 5120 slots)")
    a = ap.parse_args()
    assert "WGT" in os.environ.get("PTX_AB", "") and "wgt" in os.environ.get("PTX_LIB_PATH", ""), \
        "run with PTX_AB=WGT PTX_LIB_PATH=<libptx_wgt.so>"
    from pathtracerdemo_amd import _native as N
    from pathtracerdemo_amd.renderer import Renderer
    from pathtracerdemo_amd.scene.world import compile_scene
    lib = N.load()
    lib.ptx_diag_wave_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.ptx_diag_wave_times.restype = ctypes.c_int
    r = Renderer(a.width, a.height, device=0, pipeline=a.pipeline, single_stream=a.single_stream)
    r.Initialize(compile_scene(a.scene))
    for _ in range(3):
        r.Update()
        r.Render()
    buf = np.zeros((1 << 20, 4), dtype=np.uint64)
    lib.ptx_diag_wave_times(r._h, buf.ctypes.data, 1 << 20)  # drop the warm-up records
    for _ in range(a.frames):
        r.Update()
        r.Render()
    n = lib.ptx_diag_wave_times(r._h, buf.ctypes.data, 1 << 20)
    rec = buf[:n]
    t0 = rec[:, 0].min()
    s = (rec[:, 0] - t0).astype(np.float64) / 100.0  # us
    e = (rec[:, 1] - t0).astype(np.float64) / 100.0
    kid = (rec[:, 2] >> np.uint64(32)).astype(int)
    seq = kid >> 7  # (second launch sequence of a pipelined frame's back: kid | 0x80)
    kid = kid & 0x7f
    span = e.max()
    nb = int(np.ceil(span / a.bin_us))
    occ = {}
    seqocc = {}
    for k in sorted(set(kid)):
        o = np.zeros(nb)
        for si, ei in zip(s[kid == k], e[kid == k]):
            b0, b1 = int(si // a.bin_us), int(min(ei, span - 1e-9) // a.bin_us)
            if b0 == b1:
                o[b0] += (ei - si) / a.bin_us
            else:
                o[b0] += (b0 + 1 - si / a.bin_us)
                o[b0 + 1:b1] += 1.0
                o[b1] += ei / a.bin_us - b1
        occ[KIDS.get(k, str(k))] = o
    for k in sorted(set(kid)):  # per launch sequence of the back (0 / 1)
        for q in (0, 1):
            m = (kid == k) & (seq == q)
            if not m.any() or not (seq[kid == k] == 1).any():
                continue
            o = np.zeros(nb)
            for si, ei in zip(s[m], e[m]):
                b0, b1 = int(si // a.bin_us), int(min(ei, span - 1e-9) // a.bin_us)
                if b0 == b1:
                    o[b0] += (ei - si) / a.bin_us
                else:
                    o[b0] += (b0 + 1 - si / a.bin_us)
                    o[b0 + 1:b1] += 1.0
                    o[b1] += ei / a.bin_us - b1
            seqocc[f"{KIDS.get(k, str(k))}.{q}"] = o
    total = sum(occ.values())
    print(f"{a.frames} frame(s): span {span:.1f} us, {n} waves; mean resident waves {total.mean():.0f} "
          f"(chip: 1024 SIMDs; trace kernel 4/SIMD = 4096)")
    for name, o in occ.items():
        d = (e - s)[kid == [k for k, v in KIDS.items() if v == name][0]] if name in KIDS.values() else None
        msg = f"  {name:16s} wave-us {o.sum()*a.bin_us:10.0f}"
        if d is not None and len(d):
            msg += f"  waves {len(d):7d}  dur p50 {np.percentile(d,50):7.1f} p90 {np.percentile(d,90):7.1f} p99 {np.percentile(d,99):7.1f} max {d.max():7.1f} us"
        print(msg)
    if a.single_stream:  # trace launches one after another: split them at gaps in the waves' starts
        tk = [k for k, v in KIDS.items() if v == "trace"][0]
        m = kid == tk
        order = np.argsort(s[m])
        ts, te = s[m][order], e[m][order]
        cap = 256 * 4 * 5  # CUs x SIMDs x the streamed trace kernel's waves per SIMD
        launches, lo, end = [], 0, te[0]
        for i in range(1, len(ts) + 1):
            if i == len(ts) or ts[i] > end:
                launches.append((lo, i))
                if i < len(ts):
                    lo, end = i, te[i]
            else:
                end = max(end, te[i])
        print("trace launches (single stream): span, waves, fill = wave-us / (span x %d), time after the "
              "first wave end until the last (tail)" % cap)
        for lo, hi in launches:
            s0, e1 = ts[lo:hi].min(), te[lo:hi].max()
            d = te[lo:hi] - ts[lo:hi]
            first_end = te[lo:hi].min()
            p90_end = np.percentile(te[lo:hi], 90)
            print(f"  start {s0:8.1f} span {e1 - s0:7.1f} us  waves {hi - lo:6d}  fill {d.sum() / ((e1 - s0) * cap):.3f}  "
                  f"90% of waves done at {p90_end - s0:7.1f} us, last at {e1 - s0:7.1f}")
    print("timeline (resident waves per 20 us bin; T = trace, L = logic):")
    tr = occ.get("trace", np.zeros(nb))
    lg = total - tr
    for b in range(0, nb, max(1, nb // 80)):
        print(f"  {b*a.bin_us:7.0f} us  T {tr[b]:6.0f}  L {lg[b]:6.0f}  " + "#" * int(tr[b] / 64) + "." * int(lg[b] / 64))
    if a.out:
        json.dump({"span_us": span, "bin_us": a.bin_us, "occupancy": {k: v.tolist() for k, v in occ.items()},
                   "occupancy_by_sequence": {k: v.tolist() for k, v in seqocc.items()},
                   "records": rec.astype(np.int64).tolist() if n < 400000 else None}, open(a.out, "w"))


if __name__ == "__main__":
    main()
