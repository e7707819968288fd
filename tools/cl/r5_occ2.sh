# round 5: trace occupancy 4 vs 5 waves per SIMD on the moving camera and GI (measurement build)
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=TRACE_OCC=4" REPS=2 TAG=r5/occ2/cam BENCH_ARGS="--no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=TRACE_OCC=4" REPS=1 TAG=r5/occ2/gi BENCH_ARGS="--no-configs3 --workload gi" bash tools/ab_env.sh || exit 1
