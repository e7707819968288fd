# round 5: more hardware queues per process (GPU_MAX_HW_QUEUES 4 -> 8) with deeper stream use
# (measurement build): the headline and the moving camera
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB=""
for k in "GPU_MAX_HW_QUEUES=4 PTX_AB=" "GPU_MAX_HW_QUEUES=8 PTX_AB=" "GPU_MAX_HW_QUEUES=8 PTX_AB=PIPE_BACK_STREAMS=3" "GPU_MAX_HW_QUEUES=8 PTX_AB=PIPE_DEPTH=3" "GPU_MAX_HW_QUEUES=8 PTX_AB=PIPE_STREAMS=2"; do AB+="PTX_LIB_PATH=$L $k"$'\n'; done
AB="$AB" TAG=r5/hwq BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
