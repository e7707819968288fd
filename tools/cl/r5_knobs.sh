# round 5: the headline's pipelining / occupancy switches re-checked under the streamed walk
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB=""
for k in "" "PIPE_BACK_STREAMS=1" "PIPE_BACK_STREAMS=3" "PIPE_STREAMS=2" "TEMPORAL_SPLIT=0" "TRACE_OCC=4" "TRACE_OCC=6" ""; do AB+="PTX_LIB_PATH=$L PTX_AB=$k"$'\n'; done
AB="$AB" TAG=r5/knobs BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
