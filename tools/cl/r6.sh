# Round 6 GPU calls, one case per gpurun call: bash tools/cl/r6.sh <case>
# (every step is tools/gpu.sh; results under gpurun_out/r6/<case>/, copied to profiles/r6/)
set -o pipefail
G="bash tools/gpu.sh"
C=r6/$1
mkdir -p gpurun_out/$C
# configs[3]'s 8 bands at the round-5 last build's measured cut (profiles/r5/bands/last_build_recut.jsonl)
B5='[[0, 572], [572, 750], [750, 895], [895, 1059], [1059, 1281], [1281, 1534], [1534, 1778], [1778, 2160]]'
case "$1" in
first)  # the round's first build: suite, smoke, headline + C1 ReSTIR lines, shipped-library profile, bands
    $G suite $C && $G smoke $C &&
    $G bench $C reuse && $G bench $C restir --workload restir --no-configs3 &&
    $G profile $C/prof_reuse && $G bands $C bands_r5cut --world 8 --bands "$B5" ;;
prio)  # band back chain on high-priority streams (PTX_AB=BAND_PRIO=1, measurement build) vs the product
    $G bands $C base --world 8 --bands "$B5" &&
    PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so EXTRA_AB=BAND_PRIO=1 $G bands $C prio --world 8 --bands "$B5" &&
    PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so EXTRA_AB=BAND_PRIO=1 $G bands $C prio_overlap --world 8 --bands "$B5" --overlap &&
    $G bands $C base2 --world 8 --bands "$B5" ;;
w1)  # one-wave trace workgroups (PTX_AB=TRACE_W1=k, measurement build) and the spill-free shipped trace
     # kernel (dynamic / split-segment branches compiled out): GPU suites, then interleaved benches
    AB=$PWD/pathtracerdemo_amd/libptx_ab.so
    $G suite $C &&
    PTX_LIB_PATH=$AB PTX_AB=TRACE_W1=2 $G suite $C/w2 -k "parity or reuse or gi or bands or golden" &&
    for v in prod w0 w2 w4 prod w2 w1 w0; do
        if [ $v = prod ]; then $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1
        else PTX_LIB_PATH=$AB PTX_AB=TRACE_W1=${v#w} $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1; fi
    done &&
    for v in prod w0 w2 w4; do
        if [ $v = prod ]; then $G bench $C restir_$v --workload restir --no-cpu-baseline || exit 1
        else PTX_LIB_PATH=$AB PTX_AB=TRACE_W1=${v#w} $G bench $C restir_$v --workload restir --no-cpu-baseline || exit 1; fi
    done &&
    $G bands $C bands_prod --world 8 --bands "$B5" &&
    PTX_LIB_PATH=$AB EXTRA_AB=TRACE_W1=2 $G bands $C bands_w2 --world 8 --bands "$B5" &&
    PTX_LIB_PATH=$AB EXTRA_AB=TRACE_W1=4 $G bands $C bands_w4 --world 8 --bands "$B5" ;;
occ)  # the streamed trace kernel at 6 / 7 waves per SIMD now that the A/B batch paths are compiled out
      # (80 VGPRs + 20 B/lane spilled at 6, 72 + 60 B at 7; round 5: 6 waves spilled 136 B and lost 12 %):
      # variant build libptx_o6.so (measurement switches on, trace A/B paths off), PTX_AB=TRACE_OCC=n
    O6=$PWD/pathtracerdemo_amd/libptx_o6.so
    PTX_LIB_PATH=$O6 PTX_AB=TRACE_OCC=6 $G suite $C/o6 -k "parity or reuse or gi or golden" &&
    for v in 6 5 7 6 5; do PTX_LIB_PATH=$O6 PTX_AB=TRACE_OCC=$v $G bench $C reuse_o$v --no-cpu-baseline --no-configs3 || exit 1; done &&
    $G bench $C reuse_prod --no-cpu-baseline --no-configs3 &&
    for v in 6 5; do PTX_LIB_PATH=$O6 PTX_AB=TRACE_OCC=$v $G bench $C restir_o$v --workload restir --no-cpu-baseline || exit 1; done &&
    for v in 6 5; do PTX_LIB_PATH=$O6 PTX_AB=TRACE_OCC=$v $G bench $C gi_o$v --workload gi --no-cpu-baseline || exit 1; done &&
    for v in 6 5; do PTX_LIB_PATH=$O6 PTX_AB=TRACE_OCC=$v $G bench $C mcpt_o$v --workload mcpt --no-cpu-baseline || exit 1; done &&
    for v in 6 5; do PTX_LIB_PATH=$O6 PTX_AB=TRACE_OCC=$v $G bench $C k4_o$v --frame 3840x2160 --no-cpu-baseline || exit 1; done &&
    PTX_LIB_PATH=$O6 EXTRA_AB=TRACE_OCC=6 $G bands $C bands_o6 --world 8 --bands "$B5" ;;
tail)  # per-wave timing of the launch-timed region (diagnostic build libptx_wgt.so): how full each trace
       # launch keeps the chip, 1080p reuse / C1 ReSTIR and the 4K frame
    W=$PWD/pathtracerdemo_amd/libptx_wgt.so
    PTX_AB=WGT PTX_LIB_PATH=$W timeout -k 10 300 python -u tools/wave_timeline.py --single-stream > gpurun_out/$C/reuse.txt 2>&1 &&
    PTX_AB=WGT PTX_LIB_PATH=$W timeout -k 10 300 python -u tools/wave_timeline.py --single-stream --pipeline restir --scene dummy_scene_1 > gpurun_out/$C/restir.txt 2>&1 &&
    PTX_AB=WGT PTX_LIB_PATH=$W timeout -k 10 300 python -u tools/wave_timeline.py --single-stream --width 3840 --height 2160 > gpurun_out/$C/reuse4k.txt 2>&1 &&
    grep -A12 "trace launches" gpurun_out/$C/*.txt ;;
fused)  # the spatial pass's {trace, step} rounds as ONE launch (wspatial_rounds; PTX_AB=SPATIAL_FUSED=1, band
        # handles only with =2): variant build libptx_fu.so (switches on, trace A/B paths off) -- the reuse /
        # band / loopback GPU tests under it, then the headline and configs[3]'s bands against fused = 0
    FU=$PWD/pathtracerdemo_amd/libptx_fu.so
    PTX_LIB_PATH=$FU PTX_AB=SPATIAL_FUSED=1 $G suite $C/f1 -k "reuse or bands or loopback or golden or parity" &&
    for v in 1 0 1 0; do PTX_LIB_PATH=$FU PTX_AB=SPATIAL_FUSED=$v $G bench $C reuse_f$v --no-cpu-baseline --no-configs3 || exit 1; done &&
    for v in 1 0; do PTX_LIB_PATH=$FU PTX_AB=SPATIAL_FUSED=$v $G bench $C k4_f$v --frame 3840x2160 --no-cpu-baseline || exit 1; done &&
    PTX_LIB_PATH=$FU EXTRA_AB=SPATIAL_FUSED=2 $G bands $C bands_f2 --world 8 --bands "$B5" &&
    PTX_LIB_PATH=$FU EXTRA_AB=SPATIAL_FUSED=0 $G bands $C bands_f0 --world 8 --bands "$B5" ;;
dyn)  # dynamic trace batches with the workgroup cap of the 5-wave trace (PTX_AB=TRACE_DYN=1,DYN_GROUPS=1280;
      # round 5 measured them at the 4-wave cap of 1024 workgroups) against static slots, measurement build
    AB=$PWD/pathtracerdemo_amd/libptx_ab.so
    for v in "TRACE_DYN=1,DYN_GROUPS=1280" "TRACE_DYN=0" "TRACE_DYN=1,DYN_GROUPS=1024" "TRACE_DYN=1,DYN_GROUPS=1280" "TRACE_DYN=0"; do
        PTX_LIB_PATH=$AB PTX_AB=$v $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1; done &&
    for v in "TRACE_DYN=1,DYN_GROUPS=1280" "TRACE_DYN=0"; do
        PTX_LIB_PATH=$AB PTX_AB=$v $G bench $C restir_$v --workload restir --no-cpu-baseline || exit 1; done &&
    PTX_LIB_PATH=$AB EXTRA_AB=TRACE_DYN=1,DYN_GROUPS=1280 $G bands $C bands_dyn1280 --world 8 --bands "$B5" ;;
rehearse)  # bench.py --gpus 2 on a one-GPU box (gloo + host halo, both ranks on GPU 0): the N > 1 path runs
    PTX_DIST_BACKEND=gloo PTX_FORCE_DEVICE=0 $G bench $C gpus2 --gpus 2 --halo torch --steps 3 --warmup 1 &&
    PTX_DIST_BACKEND=gloo PTX_FORCE_DEVICE=0 $G bench $C gpus2_weak --gpus 2 --halo torch --weak --steps 3 --warmup 1 ;;
verify)  # the build after the A/Bs were removed: GPU suite + smoke + the default bench line, then the tail case
    $G suite $C && $G smoke $C && $G bench $C reuse && bash tools/cl/r6.sh tail ;;
evid)  # round-6 evidence at the current build: GPU suite + smoke, then per workload the shipped-library
       # profile (tools/gpu.sh profile) and its bench line (CPU baselines, parity window, 4K one-GPU frame);
       # then the one-wave trace workgroups against the same-box product (measurement build, TRACE_W1=2)
    AB=$PWD/pathtracerdemo_amd/libptx_ab.so
    $G suite $C && $G smoke $C &&
    for wl in reuse restir; do
        $G profile $C/prof_$wl --workload $wl && $G bench $C $wl --workload $wl || exit 1
    done &&
    PTX_LIB_PATH=$AB PTX_AB=TRACE_W1=2 $G bench $C reuse_w2 --no-cpu-baseline --no-configs3 &&
    PTX_LIB_PATH=$AB PTX_AB=TRACE_W1=0 $G bench $C reuse_w0 --no-cpu-baseline --no-configs3 &&
    $G bench $C reuse_prod --no-cpu-baseline --no-configs3 &&
    PTX_LIB_PATH=$AB PTX_AB=TRACE_W1=2 $G bench $C restir_w2 --workload restir --no-cpu-baseline &&
    $G bench $C restir_prod --workload restir --no-cpu-baseline ;;
evid2)  # the other two workloads' evidence, lane use per traversal region (measurement build), the moving
        # camera, the DYN coverage run, and configs[3]'s bands (the r5 cut, one measured re-cut)
    for wl in gi mcpt; do
        $G profile $C/prof_$wl --workload $wl && $G bench $C $wl --workload $wl || exit 1
    done &&
    PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so $G simd $C reuse &&
    PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so $G simd $C restir &&
    $G bench $C camera --camera-path --no-configs3 &&
    PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so PTX_AB=TRACE_DYN=1 $G suite $C/dyn -k "parity or reuse" &&
    $G bands $C bands --world 8 --bands "$B5" --recut 1 ;;
edge)  # band frames with the edge rows' temporal combine first, the exchange leaving beside the interior
       # rows' combine (PTX_AB=EDGE_FIRST=1, measurement build): band / loopback GPU tests, then bands
       # (lost, removed: DESIGN.md §9 item 1)
    AB=$PWD/pathtracerdemo_amd/libptx_ab.so
    PTX_LIB_PATH=$AB PTX_AB=EDGE_FIRST=1 $G suite $C/e1 -k "bands or loopback or golden" &&
    $G bands $C base --world 8 --bands "$B5" &&
    PTX_LIB_PATH=$AB EXTRA_AB=EDGE_FIRST=1 $G bands $C edge1 --world 8 --bands "$B5" &&
    PTX_LIB_PATH=$AB EXTRA_AB=EDGE_FIRST=0 $G bands $C edge0 --world 8 --bands "$B5" &&
    PTX_LIB_PATH=$AB EXTRA_AB=EDGE_FIRST=1 $G bands $C edge1b --world 8 --bands "$B5" &&
    $G bands $C base2 --world 8 --bands "$B5" ;;
seeds)  # the spatial start reading a neighbour's seeds from the summaries' 8-byte seed plane instead of
        # its reservoir line: GPU suite, then the headline / 4K / bands against the previous build
        # (libptx_prev.so = the library before the change; no gain, removed: DESIGN.md §9 item 5)
    P=$PWD/pathtracerdemo_amd/libptx_prev.so
    $G suite $C &&
    for v in new prev new prev; do
        if [ $v = new ]; then $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1
        else PTX_LIB_PATH=$P $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1; fi
    done &&
    $G bench $C k4_new --frame 3840x2160 --no-cpu-baseline && PTX_LIB_PATH=$P $G bench $C k4_prev --frame 3840x2160 --no-cpu-baseline &&
    $G bench $C cam_new --camera-path --no-cpu-baseline --no-configs3 && PTX_LIB_PATH=$P $G bench $C cam_prev --camera-path --no-cpu-baseline --no-configs3 &&
    $G bands $C bands_new --world 8 --bands "$B5" && PTX_LIB_PATH=$P $G bands $C bands_prev --world 8 --bands "$B5" ;;
sq)  # where the logic kernels' wave cycles go (SQ counters, shipped library, profile region), still and moving
    $G sq $C/reuse && python3 tools/sq_table.py gpurun_out/$C/reuse/pmc_sq/run_counter_collection.csv &&
    $G profile $C/prof_cam --camera-path --no-configs3 && $G sq $C/sq_cam --camera-path --no-configs3 &&
    python3 tools/sq_table.py gpurun_out/$C/sq_cam/pmc_sq/run_counter_collection.csv ;;
camprof)  # the moving camera's kernels (profile region, shipped library) and their SQ counters
    $G profile $C/prof_cam --camera-path --no-configs3 && $G sq $C/sq_cam --camera-path --no-configs3 &&
    python3 tools/sq_table.py gpurun_out/$C/sq_cam/pmc_sq/run_counter_collection.csv ;;
motion)  # the motion start slot-major (one job per thread and iteration: 104 B/lane spilled instead of
         # 164 at 3 waves; libptx_m2.so at 2 waves, 36 B) against the previous build (libptx_prev.so)
         # (lost 1-2 %, removed: DESIGN.md §9 item 4)
    P=$PWD/pathtracerdemo_amd/libptx_prev.so; M2=$PWD/pathtracerdemo_amd/libptx_m2.so
    $G suite $C -k "reuse or motion or camera or bands or loopback or golden or parity" &&
    for v in new prev m2 new prev m2; do
        case $v in new) L= ;; prev) L=$P ;; m2) L=$M2 ;; esac
        PTX_LIB_PATH=$L $G bench $C cam_$v --camera-path --no-cpu-baseline --no-configs3 || exit 1
    done &&
    $G bench $C reuse_new --no-cpu-baseline --no-configs3 && PTX_LIB_PATH=$P $G bench $C reuse_prev --no-cpu-baseline --no-configs3 ;;
jobload)  # job_load with one assignment per field (the job no longer kept in scratch: wjob_step 32 -> 12
          # B/lane, folded spills only) against the previous build (libptx_prev.so)
    P=$PWD/pathtracerdemo_amd/libptx_prev.so
    $G suite $C -k "reuse or motion or camera or bands or loopback or golden or parity" &&
    for v in new prev new prev; do
        if [ $v = new ]; then $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1
        else PTX_LIB_PATH=$P $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1; fi
    done &&
    $G bench $C cam_new --camera-path --no-cpu-baseline --no-configs3 && PTX_LIB_PATH=$P $G bench $C cam_prev --camera-path --no-cpu-baseline --no-configs3 &&
    $G bench $C k4_new --frame 3840x2160 --no-cpu-baseline && PTX_LIB_PATH=$P $G bench $C k4_prev --frame 3840x2160 --no-cpu-baseline &&
    $G bands $C bands_new --world 8 --bands "$B5" && PTX_LIB_PATH=$P $G bands $C bands_prev --world 8 --bands "$B5" ;;
tres)  # tile-coalesced reservoir rows in the temporal combine (tres_load / tres_store) against the
       # previous build (libptx_prev.so): reuse GPU tests, per-kernel times, headline
       # (no gain, removed: DESIGN.md §9 item 5)
    P=$PWD/pathtracerdemo_amd/libptx_prev.so
    $G suite $C -k "reuse or bands or loopback or golden or parity" &&
    $G kstats $C/k_new && PTX_LIB_PATH=$P $G kstats $C/k_prev &&
    for v in new prev new prev; do
        if [ $v = new ]; then $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1
        else PTX_LIB_PATH=$P $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1; fi
    done ;;
evid3a)  # the round's last build (job_load fix): GPU suite + smoke, the headline's and C1 ReSTIR's
         # shipped-library profiles and bench lines, the headline's SQ counters
    $G suite $C && $G smoke $C &&
    for wl in reuse restir; do
        $G profile $C/prof_$wl --workload $wl && $G bench $C $wl --workload $wl || exit 1
    done &&
    $G sq $C/sq_reuse && python3 tools/sq_table.py gpurun_out/$C/sq_reuse/pmc_sq/run_counter_collection.csv ;;
evid3b)  # the same build: GI and TEST_MCPT profiles + lines, lane use (measurement build), the moving
         # camera, configs[3]'s bands
    AB=$PWD/pathtracerdemo_amd/libptx_ab.so
    for wl in gi mcpt; do
        $G profile $C/prof_$wl --workload $wl && $G bench $C $wl --workload $wl || exit 1
    done &&
    PTX_LIB_PATH=$AB $G simd $C reuse && PTX_LIB_PATH=$AB $G simd $C restir &&
    $G bench $C camera --camera-path --no-configs3 &&
    $G bands $C bands --world 8 --bands "$B5" ;;
idc)  # the streamed walk keeping an identity instance's ray transform for the next identity instance
      # (no repeated transforms / IEEE divisions) against the previous build (libptx_prev.so)
      # (lost 1-2 %, removed: DESIGN.md §9 item 2)
    P=$PWD/pathtracerdemo_amd/libptx_prev.so
    $G suite $C &&
    $G kstats $C/k_new && PTX_LIB_PATH=$P $G kstats $C/k_prev &&
    for v in new prev new prev; do
        if [ $v = new ]; then $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1
        else PTX_LIB_PATH=$P $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1; fi
    done &&
    for wl in restir gi mcpt; do
        $G bench $C ${wl}_new --workload $wl --no-cpu-baseline && PTX_LIB_PATH=$P $G bench $C ${wl}_prev --workload $wl --no-cpu-baseline || exit 1
    done ;;
rcfree)  # diagnostic upper bound (wrong results, timing only): the reconnection vertex's surface
         # reconstruction made free of memory (libptx_rcfree.so, -DPTX_DIAG_RC_FREE) against the product
    F=$PWD/pathtracerdemo_amd/libptx_rcfree.so
    $G kstats $C/k_prod && PTX_LIB_PATH=$F $G kstats $C/k_free &&
    for v in prod free prod free; do
        if [ $v = prod ]; then $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1
        else PTX_LIB_PATH=$F $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1; fi
    done ;;
rcrec)  # reconnection-vertex records (ReuseArgs::rc: x_k's surface written beside each summary, read
        # by the spatial pass's hybrid-shift jobs) against the previous build (libptx_prev.so)
        # (no gain, removed: DESIGN.md §9, after item 7)
    P=$PWD/pathtracerdemo_amd/libptx_prev.so
    $G suite $C &&
    $G kstats $C/k_new && PTX_LIB_PATH=$P $G kstats $C/k_prev &&
    for v in new prev new prev; do
        if [ $v = new ]; then $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1
        else PTX_LIB_PATH=$P $G bench $C reuse_$v --no-cpu-baseline --no-configs3 || exit 1; fi
    done &&
    $G bench $C cam_new --camera-path --no-cpu-baseline --no-configs3 && PTX_LIB_PATH=$P $G bench $C cam_prev --camera-path --no-cpu-baseline --no-configs3 &&
    $G bench $C k4_new --frame 3840x2160 --no-cpu-baseline && PTX_LIB_PATH=$P $G bench $C k4_prev --frame 3840x2160 --no-cpu-baseline &&
    $G bands $C bands_new --world 8 --bands "$B5" && PTX_LIB_PATH=$P $G bands $C bands_prev --world 8 --bands "$B5" ;;
is5)  # the PT_1 step kernel alone at 5 waves per SIMD (libptx_is5.so, -DINIT_STEP_WAVES=5: 95 VGPRs +
      # 36 B/lane spilled, against 102 VGPRs at 4) against the product: PT_1 parity, headline, C1 ReSTIR
      # (noise either way, not kept: DESIGN.md §9)
    V=$PWD/pathtracerdemo_amd/libptx_is5.so
    PTX_LIB_PATH=$V $G suite $C/is5 -k "parity or restir or reuse_frames" &&
    $G kstats $C/k_prod && PTX_LIB_PATH=$V $G kstats $C/k_is5 &&
    for v in prod is5 prod is5; do
        if [ $v = prod ]; then $G bench $C reuse_$v --no-cpu-baseline --no-configs3 && $G bench $C restir_$v --workload restir --no-cpu-baseline || exit 1
        else PTX_LIB_PATH=$V $G bench $C reuse_$v --no-cpu-baseline --no-configs3 && PTX_LIB_PATH=$V $G bench $C restir_$v --workload restir --no-cpu-baseline || exit 1; fi
    done ;;
pmcline)  # the default bench line with roofline.traffic measured in the run (child PMC passes)
    $G bench $C reuse && $G bench $C restir --workload restir --no-configs3 --no-cpu-baseline &&
    python3 -c "import json; [print(w, json.load(open(f'gpurun_out/$C/{w}.json'))['roofline']['traffic'], json.load(open(f'gpurun_out/$C/{w}.json'))['roofline']['traffic_source']) for w in ('reuse', 'restir')]" ;;
final)  # the round's last build: GPU suite + smoke + the default bench line + C1 ReSTIR
    $G suite $C && $G smoke $C && $G bench $C reuse && $G bench $C restir --workload restir --no-configs3 ;;
*)
    echo "unknown case $1"; exit 2 ;;
esac
