# round 5: launch-shape switches for the pipelined ReSTIR frames (C1 1080p, measurement build)
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=PIPE_DEPTH=3
PTX_LIB_PATH=$L PTX_AB=SEG_PX=512
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1024
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536" REPS=2 TAG=r5/piperestir3/ab BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_env.sh || exit 1
echo done
