#!/usr/bin/env python3
"""Benchmark: Msamples/s of the reference's per-pixel path on MI355X.

Workload (BASELINE.json configs):
  * reuse (default): configs[2], the metric's "ReSTIR DI (temporal + spatial reuse)" --
    PT_01 G-buffer -> PT_1 initial RIS -> temporal reuse -> spatial reuse -> PT_4 final
    shading, 1920x1080, 1 spp per frame, on C3 (the build-defined 32-rect-light interior,
    scenes/c3_interior_32.json).  The reuse passes are build-defined.
  * restir: Renderer_TEST's live pipeline (PT_01 -> PT_1 -> PT_4, no reuse), 1080p.
  * mcpt: TEST_MCPT brute-force path tracer (configs[1]).
  * gi: configs[4], ReSTIR GI -- G-buffer -> GI init (direct light + 1-bounce indirect
    candidate) -> temporal -> spatial (reconnection shift) -> GI shade, C3, 1080p
    (build-defined).
  restir / mcpt default to DUMMY_SCENE_1 (Cornell-style room, 22 294 triangles, 3 lights).
A step = one frame (all passes) over the whole band; inputs (scene, uniform) are resident
in HBM before the timed region.

Multi-GPU (`--gpus N`, N > 1): configs[3] by default -- the C3 reuse frame at 3840x2160
split into N row bands (strong scaling), one process per GPU.  Under torchrun the ranks come
from the environment; started directly, bench.py spawns the N ranks itself (before anything
touches a GPU) and exits with their status.  Each rank takes a work census of the full frame
(counting build, PTX_FLAG_ROW_CENSUS), cuts cost-balanced bands from it
(pathtracerdemo_amd/bands.py), and renders its band through a handle that owns an RCCL
communicator: the spatial-reuse halo (reuse_radius rows of G-buffer + reservoirs to and from
the neighbouring bands) moves by grouped ncclSend/ncclRecv on the handle's stream every
frame, no host wait (pathtracerdemo_amd/csrc/ptx_comm.cpp).  `--weak` keeps the per-GPU frame
fixed instead (rank r renders rows [r*H, (r+1)*H) of a W x (H*N) frame).  Timing: barrier +
max-reduce of the elapsed time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)
L2_PEAK_GBS = 34500.0  # MI355X L2, all 8 XCDs (MI355X_MICROARCH.md §L2: ~34.5 TB/s)
# the wavefront queue's own IO per traced query (32 B ray record read + 32 B hit record
# written): layout-specific, so NOT in SURVEY §8(d)'s B_ray -- reported beside the roofline
QUEUE_IO_PER_RAY = 64
# algorithmic bytes: 32 per slab test, 36 per triangle test, 48 per
# instance transform, 48 per hit reconstruction; per-pixel pass IO below.
B_AABB, B_TRI, B_INST, B_HIT = 32, 36, 48, 48
PASS_IO = {"gbuffer": 16, "init": 16 + 128, "final": 16 + 128 + 16 + 16, "mcpt": 16 + 16,
           # temporal: G-buffer, PT_1 reservoir, history in; reservoir out.  spatial: G-buffer +
           # reservoir of the pixel and its 3 neighbours in, PT_4's reservoir out
           "temporal": 16 + 128 + 128 + 128, "spatial": 4 * (16 + 128) + 128}
# GI passes: init reads the G-buffer, writes a 64-byte GI reservoir + 16 B direct light;
# temporal reads G-buffer, reservoir, history, writes the reservoir; spatial reads the
# G-buffer + reservoir of the pixel and its 3 neighbours, writes the output; final reads
# G-buffer, output, direct light, accum and writes accum
PASS_IO_GI = {"gbuffer": 16, "init": 16 + 64 + 16, "temporal": 16 + 64 + 64 + 64, "spatial": 4 * (16 + 64) + 64,
              "final": 16 + 64 + 16 + 16 + 16}
PASSES = {"restir": ["gbuffer", "init", "final"], "mcpt": ["mcpt"],
          "reuse": ["gbuffer", "init", "temporal", "spatial", "final"],
          "gi": ["gbuffer", "init", "temporal", "spatial", "final"]}
DEFAULT_SCENE = {"reuse": "c3_interior_32", "restir": "dummy_scene_1", "mcpt": "dummy_scene_1",
                 "gi": "c3_interior_32"}


def usable_cpus() -> int:
    """CPUs this process can actually use: its affinity set, capped by the cgroup CPU quota
    (a container's share -- the GPU box shows 256 logical CPUs but allows 16)."""
    import math
    h = host_cpus()
    n = h.get("affinity") or h.get("logical") or 1
    q = h.get("cgroup_cpus")
    if q:
        n = min(n, max(1, math.ceil(q)))
    return max(1, n)


def camera_pose(step: int):
    """`--camera-path`: the camera of frame `step` (0-based) -- an interactive walk through the
    room as WebGPUEngine drives it (InputController.ts:81-159: 5 units/s at 60 Hz, i.e. ~0.08
    units per frame, with a slow mouse turn): (location, yaw in degrees)."""
    import math
    a = 0.166 * step
    return (0.5 * math.sin(a), 0.0, 6.0 - 0.3 * (1.0 - math.cos(a))), 6.0 * math.sin(0.1 * step)


def set_pose(r, step: int):
    loc, yaw = camera_pose(step)
    r.GetCamera().set_location(*loc)
    r.GetCamera().set_yaw(yaw)


def ray_bytes(c: dict) -> int:
    return B_AABB * c["aabb_tests"] + B_TRI * c["tri_tests"] + B_INST * c["instance_xforms"] + B_HIT * c["hits"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each; default 1, or WORLD_SIZE under torchrun); spawned by bench.py "
                         "itself unless run under torchrun")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["reuse", "restir", "mcpt", "gi"], default="reuse")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frame", default=None,
                    help="strong scaling: one fixed WxH frame split into row bands over the ranks "
                         "(default with --gpus > 1: 3840x2160, configs[3]); at N = 1 the frame is "
                         "--width x --height (configs[2])")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling instead: every rank renders --width x --height rows of a taller frame")
    ap.add_argument("--bands", choices=["balanced", "equal"], default="balanced",
                    help="strong scaling: band boundaries from the GPU work census, or equal heights")
    ap.add_argument("--halo", choices=["rccl", "torch"], default="rccl",
                    help="halo exchange: the handle's own RCCL communicator, or torch.distributed "
                         "(host-driven, the CPU tests' path)")
    ap.add_argument("--no-calibrate", dest="calibrate", action="store_false",
                    help="strong scaling: keep the census bands (default: re-cut them from each band's "
                         "measured frame time, untimed, before the run)")
    ap.add_argument("--halo-overlap", action="store_true",
                    help="spatial pass of the interior rows while the halo is in flight")
    ap.add_argument("--scene", default=None, help="default: c3_interior_32 (reuse), dummy_scene_1 (others)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="C-oracle CPU baseline threads (default: the CPUs this process may use -- affinity "
                         "capped by the cgroup quota; a run on every logical CPU is reported beside it)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs3", action="store_true", help="skip the configs3_one_gpu line (profiling runs)")
    ap.add_argument("--camera-path", action="store_true",
                    help="move the camera every frame (camera_pose: 5 units/s at 60 Hz and a turn), so the "
                         "temporal pass reprojects its history (the interactive case behind the UI)")
    ap.add_argument("--variant", choices=["wave", "simple"], default="wave",
                    help="kernel variant (A/B): wavefront queues, or 1 thread/pixel")
    ap.add_argument("--no-pmc-traffic", action="store_true",
                    help="skip the in-run PMC passes that measure roofline.traffic (one GPU): take the traffic "
                         "of profiles/hbm_traffic.json instead")
    ap.add_argument("--profile-region", action="store_true",
                    help="run ONLY the launch-timed region (one launch sequence, one frame in flight) on the "
                         "shipped library: what rocprofv3 profiles, so its per-kernel averages are the line's "
                         "(tools/profile.sh); no headline region, no CPU baseline")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` outside torchrun: start N rank processes of this script (nothing in
    this process has touched a GPU) and return their worst exit status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def census(cs, W, H, pipeline, device, passes):
    """GPU work census of the full W x H frame (counting build, PTX_FLAG_ROW_CENSUS): frame 1,
    then frame 2 (history valid, as in the timed region) pass by pass; per pass the (tile rows,
    5) counters {rays, instance transforms, AABB tests, triangle tests, hits} of ptx_row_census."""
    from pathtracerdemo_amd import _native as N
    from pathtracerdemo_amd.renderer import Renderer
    pid = {"gbuffer": N.PTX_PASS_GBUFFER, "init": N.PTX_PASS_INIT, "final": N.PTX_PASS_FINAL,
           "mcpt": N.PTX_PASS_MCPT, "temporal": N.PTX_PASS_TEMPORAL, "spatial": N.PTX_PASS_SPATIAL}
    rc = Renderer(W, H, device=device, pipeline=pipeline, row_census=True)
    rc.Initialize(cs)
    rc.Update()
    rc.Render()
    rc.Update()
    out = {}
    for p in passes:
        rc.reset_stats()
        rc.run_pass(pid[p])
        out[p] = rc.row_census().astype(np.float64)
    rc.close()
    return out


def calibrate_band(cs, W, H, pipeline, device, row_begin, row_end, passes, frames=4, overlap=False):
    """ms per frame of rows [row_begin, row_end) rendered alone on this rank's GPU: the band
    handle renders its frames exactly as a rank does (pipelined band frames, same launches) but
    without the halo exchange (PTX_FLAG_HALO_SKIP), after two untimed frames -- the measured band
    cost the strong split is re-cut from (bands.recalibrated_costs)."""
    from pathtracerdemo_amd.renderer import Renderer
    r = Renderer(W, H, device=device, pipeline=pipeline, row_begin=row_begin, row_end=row_end,
                 halo_overlap=overlap, halo_skip=(row_begin, row_end) != (0, H))
    r.Initialize(cs)
    t0 = 0.0
    for it in range(2 + frames):
        if it == 2:
            r.synchronize()
            t0 = time.perf_counter()
        r.Update()
        r.Render()
    r.synchronize()
    ms = (time.perf_counter() - t0) / frames * 1e3
    r.close()
    return ms


# the timed traversal symbol (every workload since round 5: the flattened walk at 5 waves per SIMD;
# GI's closest-hit instance, not its any-hit one)
TIMED_SYMBOL = "trace_queue<false, 5, false, true, false, true"


def pmc_traffic(args, W, H):
    """roofline.traffic measured in this run: two rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE:
    one pass cannot hold both) over the launch-timed region of the same workload, each a child process
    of this one (`bench.py --profile-region`), per launch of TIMED_SYMBOL: 2 * FETCH_SIZE + WRITE_SIZE
    bytes (the gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md §HBM; tools/hbm_traffic.py).
    Returns (bytes per launch, dispatches) or (None, why not)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 is not on PATH"
    child = [sys.executable, os.path.abspath(__file__), "--workload", args.workload, "--scene", args.scene,
             "--frame", f"{W}x{H}", "--variant", args.variant, "--profile-region", "--steps", "5", "--warmup", "1",
             "--no-pmc-traffic"] + (["--camera-path"] if args.camera_path else [])
    tmp = tempfile.mkdtemp(prefix="ptx_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            print(f"bench.py: in-run PMC pass {ctr}", file=sys.stderr, flush=True)
            out = os.path.join(tmp, ctr)
            cmd = ["timeout", "-s", "KILL", "180", exe, "--pmc", ctr, "-d", out, "-o", "run", "--output-format", "csv",
                   "--"] + child
            rc = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL).returncode
            if rc != 0:
                return None, f"rocprofv3 --pmc {ctr} exited {rc}"
            xs = []
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for r in csv.DictReader(fh):
                        if TIMED_SYMBOL in r["Kernel_Name"] and r["Counter_Name"] == ctr:
                            xs.append(float(r["Counter_Value"]) * 1024.0)
            if not xs:
                return None, f"no {ctr} samples of {TIMED_SYMBOL}"
            vals[ctr] = (sum(xs) / len(xs), len(xs))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return 2.0 * vals["FETCH_SIZE"][0] + vals["WRITE_SIZE"][0], vals["FETCH_SIZE"][1]


def band_work(tile_census: np.ndarray, row_begin: int, row_end: int) -> dict:
    """The counters of rows [row_begin, row_end) from a full-frame tile-row census (a tile row
    cut by the band counts by its share of rows)."""
    T = tile_census.shape[0]
    frac = np.clip(np.minimum(np.arange(1, T + 1) * 8, row_end) - np.maximum(np.arange(T) * 8, row_begin), 0, 8) / 8.0
    tot = frac @ tile_census
    keys = ("rays", "instance_xforms", "aabb_tests", "tri_tests", "hits")
    return {k: int(round(v)) for k, v in zip(keys, tot)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is None:  # under torchrun the launcher's world size is the GPU count
        args.gpus = world
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    args.scene = args.scene or DEFAULT_SCENE[args.workload]
    if world > 1 and not args.weak and not args.frame:
        args.frame = "3840x2160"  # configs[3]
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # rehearsal knobs for one-GPU boxes: PTX_DIST_BACKEND=gloo (host halo messages) and
    # PTX_FORCE_DEVICE=0 (every rank on GPU 0); the real run is nccl (RCCL), one GPU per rank
    backend = os.environ.get("PTX_DIST_BACKEND", "nccl")
    device = int(os.environ.get("PTX_FORCE_DEVICE", local_rank))
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(device)
        dist.init_process_group(backend=backend)

    from pathtracerdemo_amd.renderer import Renderer
    from pathtracerdemo_amd.scene.world import compile_scene
    from pathtracerdemo_amd import bands as B

    cs = compile_scene(args.scene)
    pipeline = args.workload
    passes = PASSES[pipeline]
    strong = bool(args.frame) and not args.weak
    if strong:  # configs[3]: the ranks share one frame
        W, H = (int(v) for v in args.frame.lower().split("x"))
    else:  # weak scaling: rank r renders rows [r*Hb, (r+1)*Hb) of a W x (Hb*N) frame
        W, H = args.width, args.height * world
    # work census of the exact frame (counting build, untimed): algorithmic bytes, and the
    # cost-balanced bands of a strong-scaled frame
    cen = census(cs, W, H, pipeline, device, passes)
    radius = 30
    calib = None
    if strong and world > 1:
        if args.bands == "balanced":
            total = sum(cen.values())
            costs = B.row_costs(total, W, H)
            all_bands = B.balanced_bands(costs, world, min_rows=radius)
        else:
            all_bands = [B.band(H, world, r) for r in range(world)]
            costs = B.row_costs(sum(cen.values()), W, H)
        balance = B.band_balance(costs, all_bands)
        if args.bands == "balanced" and args.calibrate and dist is not None:
            # time every rank's band alone (no exchange), gather, rescale the row costs by
            # measured / predicted band cost and cut again (bands.recalibrated_costs); a band's
            # time is not additive in its rows (per-band launch tails), so four measured rounds,
            # 10 frames each, and the split keeps the measured cut with the smallest largest band
            # (a re-cut is a prediction; the measured cut of the last round can be the better one)
            calib = {"rounds": []}
            best = None
            for _ in range(4):
                b0, b1 = all_bands[rank]
                cal = calibrate_band(cs, W, H, pipeline, device, b0, b1, passes, frames=10,
                                     overlap=args.halo_overlap)
                gathered = [None] * world
                dist.all_gather_object(gathered, cal)
                calib["rounds"].append({"bands": [list(b) for b in all_bands],
                                        "band_ms": [round(v, 4) for v in gathered],
                                        "measured_max_over_mean": round(max(gathered) / (sum(gathered) / world), 4)})
                if best is None or max(gathered) < best[0]:
                    best = (max(gathered), [list(b) for b in all_bands], costs)
                costs = B.recalibrated_costs(costs, all_bands, gathered)
                all_bands = B.balanced_bands(costs, world, min_rows=radius)
            _, all_bands, costs = best
            all_bands = [tuple(b) for b in all_bands]
            calib["chosen_round"] = [r["bands"] for r in calib["rounds"]].index([list(b) for b in all_bands])
            balance = B.band_balance(costs, all_bands)
    else:
        all_bands = [B.weak_band(H // world, r) for r in range(world)]
        balance = 1.0
    row_begin, row_end = all_bands[rank]
    Hb = row_end - row_begin
    reuse = pipeline in ("reuse", "gi")
    use_comm = reuse and world > 1 and args.halo == "rccl"
    comm_fallback = None  # why the RCCL halo was not used, when rank 0 could not create an id

    def make(**kw):
        nonlocal use_comm, comm_fallback
        r = Renderer(W, H, device=device, pipeline=pipeline, row_begin=row_begin, row_end=row_end,
                     variant=args.variant, halo_overlap=args.halo_overlap, **kw)
        r.Initialize(cs)
        drv = None
        if use_comm:  # the handle's own RCCL communicator: ptx_render exchanges the halo
            # rank 0 creates the id; if it cannot (no RCCL to open), every rank learns it from
            # the broadcast and drives the halo over torch.distributed instead -- together, so
            # no rank waits in a communicator init its peers never join (reported in the line)
            uid, err = None, None
            if rank == 0:
                try:
                    uid = Renderer.comm_unique_id()
                except Exception as e:  # noqa: BLE001 -- any failure selects the fallback
                    err = f"{type(e).__name__}: {e}"
            obj = [(uid, err)]
            dist.broadcast_object_list(obj, src=0)
            uid, err = obj[0]
            if uid is not None:
                r.comm_init(uid, rank, world)
            else:
                use_comm, comm_fallback = False, err
        if not use_comm and reuse and world > 1:
            if args.camera_path:  # (every rank takes this branch together: the fallback is broadcast)
                raise SystemExit("--camera-path needs the handles' RCCL halo: the torch.distributed band "
                                 "driver (bands.ReuseBand) drops the history on a camera move")
            from pathtracerdemo_amd.bands import ReuseBand
            drv = ReuseBand(r, rank, world, device=f"cuda:{device}" if backend == "nccl" else "cpu")
        return r, drv

    if args.profile_region:
        args.no_cpu_baseline = args.no_configs3 = True
    r, band_drv = (None, None) if args.profile_region else make()

    steps_done = {}

    def frame(rr, drv):
        if args.camera_path:  # every handle walks the same path from its own first frame
            k = steps_done.get(id(rr), 0)
            steps_done[id(rr)] = k + 1
            set_pose(rr, k)
        rr.Update()
        if drv is None:
            rr.Render()
        else:
            drv.render_frame()

    from pathtracerdemo_amd import _native as N
    pid = {"gbuffer": N.PTX_PASS_GBUFFER, "init": N.PTX_PASS_INIT, "final": N.PTX_PASS_FINAL,
           "mcpt": N.PTX_PASS_MCPT, "temporal": N.PTX_PASS_TEMPORAL, "spatial": N.PTX_PASS_SPATIAL}
    counts = {p: band_work(cen[p], row_begin, row_end) for p in passes}
    px = W * Hb
    pio = PASS_IO_GI if pipeline == "gi" else PASS_IO
    alg_bytes = {p: ray_bytes(counts[p]) + pio[p] * px for p in passes}

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(rr, drv):
        """W untimed warmup frames, then K frames between barriers + synchronize: seconds."""
        for _ in range(args.warmup):
            frame(rr, drv)
        rr.synchronize()
        rr.reset_stats()
        barrier()
        rr.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            frame(rr, drv)
        rr.synchronize()
        barrier()
        return time.perf_counter() - t0

    band_digest = comm = None
    motion_clips = None
    frames_rendered = args.warmup + args.steps
    if r is not None:
        elapsed = timed(r, band_drv)
        own_elapsed = elapsed
        if dist is not None:
            import torch
            t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}" if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        st = r.stats()
        img = r.read_image()
        nonfinite = int((~np.isfinite(img[..., :3])).sum())
        if args.camera_path and reuse:
            # pixels of the timed frames whose reprojection fell outside the rows the handle holds
            # (the global motion row rule: more than reuse_radius rows from the pixel's own row)
            motion_clips = r.read_counters()["motion_clips"]
        # multi-rank self-check: each rank's band (radiance + spatial output after every frame it
        # rendered) is hashed here and compared on rank 0 with the same rows of ONE handle of the
        # whole frame rendered the same number of frames (bands are bit-identical by design)
        if reuse and world > 1 and strong:
            import hashlib
            band_digest = hashlib.sha256(img.tobytes() + r.read_history().tobytes()).hexdigest()
        comm = r.comm_info() if use_comm else None
        r.close()

    # Second timed region, same K steps, with HIP events around every wavefront launch
    # (PTX_FLAG_TIME_LAUNCHES costs ~5% of a frame, so the headline region above runs
    # without them): per-launch durations of the dominant kernel for the roofline.  It runs
    # as ONE launch sequence (PTX_FLAG_SINGLE_STREAM): in the multi-stream production frame
    # kernels share the GPU and a launch's duration measures the share, not the kernel;
    # the overlap's gain is in `value` and in roofline.frame.
    st_k = None
    if args.variant == "wave":
        rk, drv_k = make(time_launches=True, single_stream=True)
        args.warmup = max(1, args.warmup)
        el_k = timed(rk, drv_k)
        st_k = rk.stats()
        if r is None:  # --profile-region: this region is the run
            elapsed = own_elapsed = el_k
            st = st_k
            img = rk.read_image()
            nonfinite = int((~np.isfinite(img[..., :3])).sum())
        rk.close()

    # per-rank band times, communicators and band digests (rank 0 reports them all)
    band_ms = [own_elapsed / args.steps * 1e3]
    ranks_info = None
    if dist is not None:
        import torch
        t = torch.zeros(world, dtype=torch.float64, device=f"cuda:{device}" if backend == "nccl" else "cpu")
        t[rank] = own_elapsed / args.steps * 1e3
        dist.all_reduce(t)
        band_ms = [round(float(v), 4) for v in t.tolist()]
        ranks_info = [None] * world
        dist.all_gather_object(ranks_info, {"rank": rank, "device": device, "rows": [row_begin, row_end],
                                            "comm": comm, "digest": band_digest})
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    parity = None
    if band_digest is not None:
        parity = one_handle_check(cs, W, H, pipeline, device, frames_rendered, ranks_info, args.camera_path)
    samples = W * H * args.steps  # all ranks, 1 spp
    value = samples / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3
    if st["kernel_launches"][N.PTX_STAT_FRAME]:
        # the wavefront frame overlaps its passes on several streams: timed as a whole.  A
        # whole-image reuse handle pipelines its frames (two in flight: frame N's G-buffer +
        # PT_1 beside frame N-1's spatial pass), so one frame's event span overlaps the next
        # one's: the frame's GPU time is then the wall-clock time per frame
        span = st["kernel_ms_total"][N.PTX_STAT_FRAME] / st["kernel_launches"][N.PTX_STAT_FRAME]
        kms = {"frame": min(span, ms_per_step)}
        if span > 1.05 * ms_per_step:
            kms["frame_event_span"] = span
    elif st["kernel_launches"][N.PTX_STAT_PASS_GROUP]:
        # a reuse band driven from Python: two pass groups around the halo exchange, per frame
        kms = {"pass_groups": st["kernel_ms_total"][N.PTX_STAT_PASS_GROUP] / args.steps}
    else:
        kms = {p: st["kernel_ms_total"][pid[p]] / max(1, st["kernel_launches"][pid[p]]) for p in passes}
    # frame-level figure of SURVEY.md §8d: algorithmic bytes of the frame / kernel time
    frame_bytes = sum(alg_bytes.values())
    frame_kernel_s = sum(v for k, v in kms.items() if k != "frame_event_span") * 1e-3
    n_trace = st_k["kernel_launches"][N.PTX_STAT_WAVE_TRACE] if st_k else 0
    if n_trace:
        # wavefront: the dominant kernel is trace_queue (every trace round of every pass).
        # Its algorithmic bytes per launch = the frame's traversal bytes (+ 32 B ray record
        # read and 32 B hit record written per query) / trace launches per frame; its
        # duration is the HIP-event average over the timed region.
        dom = "trace_queue"
        traced = [p for p in passes if p != "gbuffer"]
        if st_k["kernel_launches"][N.PTX_STAT_FINAL_FUSED]:
            # the library reports that the reuse pipeline's PT_4 walked its replays inside its one
            # logic kernel (wfinal_one): none of its queries reached trace_queue
            traced = [p for p in traced if p != "final"]
        work = {k: sum(counts[p][k] for p in traced) for k in counts[traced[0]]}
        per_frame = n_trace / args.steps
        # SURVEY §8(d)'s B_ray only (layout-neutral); the queue's 64 B per query beside it
        dom_bytes = ray_bytes(work) / per_frame
        queue_io = QUEUE_IO_PER_RAY * work["rays"] / per_frame
        dom_ms = st_k["kernel_ms_total"][N.PTX_STAT_WAVE_TRACE] / n_trace
        logic_ms = (st_k["kernel_ms_total"][N.PTX_STAT_WAVE_LOGIC]
                    / max(1, st_k["kernel_launches"][N.PTX_STAT_WAVE_LOGIC]))
        extra = {"launches_per_frame": per_frame, "logic_kernel_avg_ms": round(logic_ms, 4),
                 "queue_io_bytes_per_launch": int(queue_io),
                 "frac_with_queue_io": round((dom_bytes + queue_io) / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 "bytes_note": "alg_bytes_per_launch = SURVEY §8(d) B_ray (32 per AABB test + 36 per triangle test "
                               "+ 48 per instance transform + 48 per hit reconstruction) / trace launches per frame; "
                               "the wavefront queue's own ray / hit records (64 B per query) are NOT counted in frac"}
    else:
        dom = max(kms, key=lambda p: kms[p])
        work = counts[dom]
        dom_bytes = alg_bytes[dom]
        dom_ms = kms[dom]
        extra = {}
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    limiters = None
    # (profiles/hbm_traffic.json and profiles/limiters.json travel to the GPU box: .gpurunignore
    # excludes only the per-round profile directories)
    key = f"{pipeline}:{args.scene}:{dom}:{W}x{Hb}"
    prof = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    traffic_source = None
    if os.path.exists(prof):
        try:
            entry = json.load(open(prof)).get(key)
            traffic = entry["bytes_per_launch"] if isinstance(entry, dict) else entry
            if traffic:
                traffic_source = ("profiles/hbm_traffic.json (" + (entry.get("source", "?") if isinstance(entry, dict)
                                                                   else "?") + "): an earlier run's PMC passes")
        except Exception:
            traffic = None
    # measured in this run where the box allows it (one GPU, the timed traversal symbol)
    if (world == 1 and n_trace and args.variant == "wave" and not args.profile_region
            and not args.no_pmc_traffic):
        measured, info = pmc_traffic(args, W, Hb)
        if measured is not None:
            traffic = int(round(measured))
            traffic_source = (f"measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (child "
                              f"processes, launch-timed region, {info} dispatches), 2*FETCH_SIZE + WRITE_SIZE per "
                              f"launch of {TIMED_SYMBOL}>")
        elif traffic_source:
            traffic_source += f"; in-run PMC unavailable: {info}"
        else:
            traffic_source = f"in-run PMC unavailable: {info}"
    lim = os.path.join(ROOT, "profiles", "limiters.json")
    if os.path.exists(lim) and n_trace:
        try:
            entry = json.load(open(lim)).get(key)
        except Exception:
            entry = None
        if entry:
            # what bounds the kernel: the L2's request bytes against its peak, and the
            # lanes the traversal's node loop keeps busy (the simd_util build)
            limiters = dict(entry)
            l2 = entry.get("l2_bytes_per_launch")
            if l2:
                limiters["l2_achieved_gbs"] = round(l2 / (dom_ms * 1e-3) / 1e9, 1)
                limiters["l2_peak_gbs"] = L2_PEAK_GBS
                limiters["l2_frac"] = round(l2 / (dom_ms * 1e-3) / 1e9 / L2_PEAK_GBS, 4)
            if traffic:
                limiters["hbm_traffic_frac"] = round(traffic / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    cpu = ts_cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(cs, W, Hb, pipeline, args.cpu_threads or usable_cpus(), device=device,
                           camera_path=args.camera_path)
        ts_cpu = ts_cpu_baseline(cs, args.scene, W, Hb, args.cpu_threads or usable_cpus(), rows=Hb)
    # configs[3]'s 3840x2160 frame on this one GPU: the single-GPU reference of the strong
    # split the N > 1 lines run (their per-GPU efficiency is value_N / (N x this value))
    one_gpu_4k = None
    if world == 1 and pipeline == "reuse" and (W, H) == (1920, 1080) and args.variant == "wave" and not args.no_configs3:
        one_gpu_4k = one_gpu_rate(cs, 3840, 2160, pipeline, device, max(5, args.steps // 2), args.warmup)
    if world > 1:
        workload = (f"{args.scene} {pipeline} {W}x{H} split over {world} GPUs, 1 spp/frame (configs[3])"
                    if strong else f"{args.scene} {pipeline} {W}x{Hb} per GPU, 1 spp/frame")
    else:
        workload = f"{args.scene} {pipeline} {W}x{H}, 1 spp/frame" + (" (configs[2])" if pipeline == "reuse" and
                                                                        (W, H) == (1920, 1080) else "")
    if args.camera_path:
        workload += ", camera moving every frame (bench.camera_pose: 5 units/s at 60 Hz + a turn; history reprojected)"
    line = {
        "metric": "Msamples/sec at 1920x1080, 1 spp ReSTIR DI; per-pixel L2 vs WebGPU ref",
        "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong" if strong or world == 1 else "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": workload,
                   "pipeline": {"restir": "PT_01 gbuffer -> PT_1 init -> PT_4 final",
                                "reuse": "PT_01 gbuffer -> PT_1 init -> temporal -> spatial (3 neighbours, "
                                         "radius 30, pairwise MIS) -> PT_4 final",
                                "mcpt": "TEST_MCPT brute force",
                                "gi": "PT_01 gbuffer -> GI init (direct + 1-bounce candidate) -> temporal -> "
                                      "spatial (3 neighbours, radius 30, reconnection shift, pairwise MIS) -> "
                                      "GI shade"}[pipeline],
                   "frame": f"{W}x{H}", "band_rows_per_gpu": Hb,
                   "parallelism": f"row-bands x{world}" + (
                       f", halo over {'the handles RCCL communicators' if use_comm else 'torch.distributed'}"
                       + (" overlapped with the interior spatial pass" if args.halo_overlap else "")
                       if reuse and world > 1 else "")},
        "kernel_ms": {p: round(v, 4) for p, v in kms.items()},
        "nonfinite_px": nonfinite,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_source,
                     "avg_launch_ms": round(dom_ms, 4), "alg_bytes_per_launch": int(dom_bytes),
                     "work_per_frame": work, **extra, "limiters": limiters,
                     "frame": {"alg_bytes": int(frame_bytes), "alg_bytes_per_sample": round(frame_bytes / px, 1),
                               "kernel_ms": round(frame_kernel_s * 1e3, 4),
                               "frac": round(frame_bytes / frame_kernel_s / (HBM_PEAK_GBS * 1e9), 4)}},
        "cpu_baseline": cpu,
        "ts_cpu_baseline": ts_cpu,
    }
    if cpu is not None and "parity" in cpu:
        line["parity"] = cpu.pop("parity")
    if motion_clips is not None:
        line["motion_clip_px"] = {"pixels": int(motion_clips), "of": W * Hb * args.steps,
                                  "note": "timed frames' pixels whose reprojected history lay more than reuse_radius "
                                          "rows away (no history there: the global motion row rule, DESIGN §4.3)"}
    if args.profile_region:
        line["profile_region"] = ("launch-timed region only (one launch sequence, one frame in flight): value is "
                                  "NOT the headline throughput")
    if world == 1:
        line["scaling_note"] = ("one GPU: configs[2]'s frame; `--gpus N` splits configs[3]'s 3840x2160 frame into N "
                                "row bands (strong); configs3_one_gpu is that frame on this one GPU")
    if one_gpu_4k is not None:
        line["configs3_one_gpu"] = one_gpu_4k
    if world > 1:
        line["bands"] = {"rows": [list(b) for b in all_bands], "split": args.bands if strong else "weak",
                         "predicted_max_over_mean": round(balance, 4), "ms_per_frame_by_rank": band_ms}
        if calib is not None:
            line["bands"]["calibration"] = calib
        line["ranks"] = [{k: v for k, v in ri.items() if k != "digest"} for ri in ranks_info]
        if comm_fallback is not None:
            line["halo_fallback"] = f"torch.distributed halo: no RCCL unique id on rank 0 ({comm_fallback})"
        if parity is not None:
            line["parity_check"] = parity
    # any PTX_* switch in the environment (PTX_AB selects A/B kernel variants: unset = product)
    line["env"] = {k: v for k, v in sorted(os.environ.items()) if k.startswith("PTX_")}
    # which libptx.so ran (product / measurement build), and PTX_AB keys it ignored
    line["library"] = N.build_info()
    if line["library"].get("ptx_ab_ignored"):
        line["env_warning"] = (f"PTX_AB keys {line['library']['ptx_ab_ignored']} are not honoured by this "
                               f"{line['library']['build']} build: the line measures its defaults")
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def one_handle_check(cs, W, H, pipeline, device, frames, ranks_info, camera_path=False):
    """Rank 0, after the timed regions: ONE handle of the whole W x H frame renders `frames`
    frames (along the same camera path as the bands when `camera_path`) and the rows of every
    rank's band must hash to that rank's digest (radiance + spatial output, bit for bit)."""
    import hashlib
    from pathtracerdemo_amd.renderer import Renderer
    one = Renderer(W, H, device=device, pipeline=pipeline)
    one.Initialize(cs)
    for k in range(frames):
        if camera_path:
            set_pose(one, k)
        one.Update()
        one.Render()
    img, hist = one.read_image(), one.read_history()
    one.close()
    bad = [ri["rank"] for ri in ranks_info
           if hashlib.sha256(img[ri["rows"][0]:ri["rows"][1]].tobytes() +
                             hist[ri["rows"][0]:ri["rows"][1]].tobytes()).hexdigest() != ri["digest"]]
    return {"bands_bit_identical_to_one_handle": not bad, "ranks_differing": bad, "frames": frames,
            "compared": "radiance + spatial-output reservoirs of every band vs the same rows of one "
                        f"{W}x{H} handle on rank 0's GPU"}


def one_gpu_rate(cs, W, H, pipeline, device, steps, warmup):
    """Msamples/s of one whole W x H frame per step on this GPU (one handle, untimed census-free)."""
    from pathtracerdemo_amd.renderer import Renderer
    r = Renderer(W, H, device=device, pipeline=pipeline)
    r.Initialize(cs)
    for _ in range(warmup):
        r.Update()
        r.Render()
    r.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        r.Update()
        r.Render()
    r.synchronize()
    dt = time.perf_counter() - t0
    r.close()
    return {"frame": f"{W}x{H}", "value": round(W * H * steps / dt / 1e6, 3), "unit": "Msamples/s",
            "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps,
            "note": "configs[3]'s frame on ONE GPU: the reference for the N-GPU strong split"}


def cpu_baseline(cs, W, H, pipeline, threads, device=0, camera_path=False):
    """The C oracle (a port of the WGSL + the reuse passes) on the host cores, timed over
    whole frames: one frame (restir / mcpt), two for reuse / GI (the second with its history).

    The oracle's frames are then the checker of the benched configuration (N = 1): a fresh
    handle renders the same frames of the same frame size, camera and scene on the GPU, and
    the whole image (+ the spatial-output reservoirs for reuse) is compared with them bit for
    bit -- the line's `parity` field (relative L2 of the radiance beside it)."""
    from oracle import oracle as O
    from pathtracerdemo_amd.scene.camera import Camera
    threads = max(1, threads)
    cam = Camera(W, H)
    cam.set_location(0, 0, 6)
    u = cs.uniform(W, H, cam.view_projection_inverse(), cam.location, 1)
    nf = 2 if pipeline in ("reuse", "gi") else 1

    def pose_uniform(f):
        c = Camera(W, H)
        loc, yaw = camera_pose(f - 1)
        c.set_location(*loc)
        c.set_yaw(yaw)
        return cs.uniform(W, H, c.view_projection_inverse(), c.location, f)

    def full_frames(nthreads, rect=None):
        fr = O.Frame(pose_uniform(1) if camera_path else u, cs.scene, cs.geometry, cs.accel)
        t0 = time.perf_counter()
        for f in range(1, nf + 1):
            if camera_path:
                fr.set_camera(pose_uniform(f))
            fr.set_frame_index(f)
            if pipeline == "reuse":
                fr.run_reuse_frame(threads=nthreads, rect=rect)
            elif pipeline == "gi":
                fr.run_gi_frame(threads=nthreads, rect=rect)
            else:
                fr.run(O.PASS_RESTIR if pipeline == "restir" else O.PASS_MCPT, threads=nthreads, rect=rect)
        return time.perf_counter() - t0, fr

    dt, fr = full_frames(threads)
    logical = os.cpu_count() or 1
    dt_all = full_frames(logical)[0] if logical != threads else dt
    # one thread on a 64-row band of the same frames (the single-core rate)
    rows = min(H, 64)
    y0 = (H - rows) // 2
    dt1 = full_frames(1, rect=(0, y0, W, y0 + rows))[0]
    out = {"value": round(nf * W * H / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": f"{nf} full {W}x{H} frame(s) ({pipeline}, FrameIndex 1..{nf}), C oracle, {threads} pthreads "
                     "(the CPUs this process may use: affinity capped by the cgroup quota)",
           "seconds": round(dt, 2), "cpu_model": cpu_model(), "host_cpus": host_cpus(),
           "at_all_logical_cpus": {"value": round(nf * W * H / dt_all / 1e6, 4), "unit": "Msamples/s",
                                   "cores": logical, "seconds": round(dt_all, 2)},
           "single_thread": {"value": round(nf * W * rows / dt1 / 1e6, 4), "unit": "Msamples/s",
                             "sample": f"rows {y0}..{y0 + rows} of the same {nf} frame(s), 1 thread",
                             "seconds": round(dt1, 2)}}
    try:
        out["parity"] = frame_parity(cs, W, H, pipeline, device, nf, fr, camera_path)
    except Exception as e:  # noqa: BLE001 -- reported, never hidden
        out["parity"] = {"error": f"{type(e).__name__}: {e}"}
    return out


def frame_parity(cs, W, H, pipeline, device, nf, fr, camera_path=False):
    """The benched configuration's first `nf` frames on a fresh handle vs the oracle's frames
    `fr` (same scene, size, camera (path), FrameIndex 1..nf): bit-exactness and relative L2."""
    from pathtracerdemo_amd.renderer import Renderer
    r = Renderer(W, H, device=device, pipeline=pipeline)
    r.Initialize(cs)
    for k in range(nf):
        if camera_path:
            set_pose(r, k)
        r.Update()
        r.Render()
    img = r.read_image()
    hist = r.read_history() if pipeline == "reuse" else None
    r.close()
    want = np.asarray(fr.accum).reshape(img.shape)
    diff_px = int(np.any(img.view(np.uint32) != want.view(np.uint32), axis=-1).sum())
    a, b = img[..., :3].astype(np.float64), want[..., :3].astype(np.float64)
    den = float(np.sqrt((b * b).sum()))
    out = {"frames": nf, "pixels": W * H, "radiance_pixels_differing": diff_px,
           "rel_l2": float(np.sqrt(((a - b) ** 2).sum())) / den if den > 0 else 0.0}
    bit_exact = diff_px == 0
    if hist is not None:
        hw = np.asarray(fr.res_hist).reshape(hist.shape)
        nres = int(np.any(hist.view(np.uint32) != hw.view(np.uint32), axis=-1).sum())
        out["reservoir_pixels_differing"] = nres
        bit_exact = bit_exact and nres == 0
    out["bit_exact"] = bit_exact
    out["compared"] = ("the whole image" + (" + all 32 words of every spatial-output reservoir" if hist is not None
                                             else "") + f" of frames 1..{nf} on the GPU vs the C oracle"
                       + (" (camera moving between them)" if camera_path else ""))
    return out


def host_cpus() -> dict:
    """Logical CPUs of the host, those this process may run on, and its cgroup CPU quota (the
    share a container actually gets), so the baseline's thread count can be read against them."""
    out = {"logical": os.cpu_count()}
    try:
        out["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            out["cgroup_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return out


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip() + f" ({os.cpu_count()} logical CPUs visible)"
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def ts_cpu_baseline(cs, scene, W, H, threads, rows=None):
    """SURVEY.md §8(d)'s JS CPU tracer (pathtracerdemo_amd/js/cpu: the reference's live
    pipeline PT_01 -> PT_1 -> PT_4 restated in JavaScript, bit-identical to the oracle) on
    Node worker_threads: a band of `rows` rows in the middle of the frame, wall clock."""
    import shutil
    import subprocess
    import tempfile
    node = shutil.which("node")
    if node is None:
        return None
    from pathtracerdemo_amd.scene.camera import Camera
    from pathtracerdemo_amd.scene.export import export_compiled
    threads = max(1, min(threads, os.cpu_count() or 1))
    rows = rows or H
    cam = Camera(W, H)
    cam.set_location(0, 0, 6)
    u = cs.uniform(W, H, cam.view_projection_inverse(), cam.location, 1)
    y0 = max(0, H // 2 - rows // 2)
    y1 = min(H, y0 + rows)
    with tempfile.TemporaryDirectory() as tmp:
        d = export_compiled(cs, os.path.join(tmp, "scene"), scene)
        uf = os.path.join(tmp, "u.bin")
        np.asarray(u, dtype="<u4").tofile(uf)
        out = subprocess.run([node, os.path.join(ROOT, "pathtracerdemo_amd", "js", "cpu", "bench_cpu.js"), d, uf,
                              str(threads), str(y0), str(y1)], capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return {"error": out.stderr[-300:]}
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return {"value": round(r["msamples_per_s"], 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "language": "JavaScript (Node worker_threads, pathtracerdemo_amd/js/cpu/pt_cpu.js)",
            "sample": f"rows {y0}..{y1} of the {W}x{H} {scene} frame, PT_01 -> PT_1 -> PT_4 (the reference's "
                      f"live pipeline; no reuse passes), FrameIndex 1", "seconds": round(r["seconds"], 2)}


if __name__ == "__main__":
    main()
