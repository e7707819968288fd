# round 5: node-loop break for waiting lanes (PTX_STREAM_NODE_BREAK, libptx_nb*.so) + the
# headline's pipelining / occupancy switches under the streamed walk (measurement build)
set -o pipefail
LIBS="libptx.so libptx_nb8.so libptx_nb16.so libptx_nb32.so" REPS=2 TAG=r5/nb BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_nb16.so" REPS=1 TAG=r5/nb_gi BENCH_ARGS="--workload gi --no-configs3" bash tools/ab_libs.sh || exit 1
bash tools/cl/r5_knobs.sh || exit 1
