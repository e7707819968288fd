# hardware queues per process (HIP's GPU_MAX_HW_QUEUES, default 4) for the pipelined frame
# (front 1 + back 2 launch sequences per frame, two contexts' streams), and 3 / 4 back sequences
# with 8 queues: same-box A/B, 2 reps
set -o pipefail
AB=$'GPU_MAX_HW_QUEUES=4\nGPU_MAX_HW_QUEUES=8 PTX_AB=PIPE_BACK_STREAMS=3\nGPU_MAX_HW_QUEUES=8 PTX_AB=PIPE_BACK_STREAMS=4\nGPU_MAX_HW_QUEUES=8 PTX_AB=PIPE_STREAMS=2' REPS=2 TAG=ab_hwq BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
