# round-2 session 5: branch-free node test A/B, GI occlusion-kernel occupancy, 4K occupancy
set -o pipefail
P=$PWD/pathtracerdemo_amd
LIBS="libptx_bf.so libptx.so" PARITY=1 REPS=3 TAG=ab_bf bash tools/ab_libs.sh || exit 1
BENCH_ARGS="--workload gi" AB="PTX_TRACE_OCC=4 PTX_LIB_PATH=$P/libptx.so"$'\n'"PTX_TRACE_OCC=4 PTX_LIB_PATH=$P/libptx_occ4.so" REPS=2 TAG=occ4_gi bash tools/ab_env.sh || exit 1
BENCH_ARGS="--frame 3840x2160" STEPS=10 AB=$'PTX_TRACE_OCC=4\nPTX_TRACE_OCC=5' REPS=2 TAG=occ_4k bash tools/ab_env.sh || exit 1
