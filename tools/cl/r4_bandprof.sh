# round 4: where a 1 Mpx band's frame time goes -- rocprofv3 kernel stats of one configs[3] band
# (rows 886-1064, the rank path without the exchange) and of the one-GPU 4K frame, both one launch
# sequence and one frame in flight, so per-kernel durations compare
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PTX_AB=WAVE_STREAMS=1,PIPELINE_FRAMES=0,TRACE_DYN=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4_bandprof/band -o run --output-format csv -- \
  python3 -c "import sys; sys.path.insert(0, '$R'); import bench; from pathtracerdemo_amd.scene.world import compile_scene; cs = compile_scene('c3_interior_32'); print(bench.calibrate_band(cs, 3840, 2160, 'reuse', 0, 886, 1064, bench.PASSES['reuse'], frames=6))" > $R/gpurun_out/r4_bandprof/band.log 2>&1 || { echo "band prof failed"; tail -5 $R/gpurun_out/r4_bandprof/band.log; exit 1; }
tail -1 $R/gpurun_out/r4_bandprof/band.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4_bandprof/full -o run --output-format csv -- \
  python3 -c "import sys; sys.path.insert(0, '$R'); import bench, json; from pathtracerdemo_amd.scene.world import compile_scene; cs = compile_scene('c3_interior_32'); print(json.dumps(bench.one_gpu_rate(cs, 3840, 2160, 'reuse', 0, 6, 2)))" > $R/gpurun_out/r4_bandprof/full.log 2>&1 || { echo "full prof failed"; tail -5 $R/gpurun_out/r4_bandprof/full.log; exit 1; }
tail -1 $R/gpurun_out/r4_bandprof/full.log
