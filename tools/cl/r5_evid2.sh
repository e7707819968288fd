# round 5: C1 ReSTIR trace occupancy (measurement build), GI with the camera moving every frame,
# then the restir / mcpt evidence at this build
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=TRACE_OCC=4"$'\n'"PTX_LIB_PATH=$L PTX_AB=TRACE_OCC=4,SEG_PX=1024" \
  TAG=r5/c1occ BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_env.sh || exit 1
mkdir -p gpurun_out/r5/gicam
timeout -k 10 300 python3 bench.py --workload gi --camera-path --no-configs3 --no-cpu-baseline > gpurun_out/r5/gicam/bench.log 2>&1 || { echo "gi camera failed"; tail -5 gpurun_out/r5/gicam/bench.log; exit 1; }
tail -1 gpurun_out/r5/gicam/bench.log | cut -c1-200
ROUND=r5 WORKLOADS="restir mcpt" bash tools/round_evidence.sh || exit 1
