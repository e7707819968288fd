# round 5: pipelined ReSTIR frames -- segment size x sequences per context (C1 1080p, measurement build)
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536
PTX_LIB_PATH=$L PTX_AB=SEG_PX=2048
PTX_LIB_PATH=$L PTX_AB=SEG_PX=3072
PTX_LIB_PATH=$L PTX_AB=SEG_PX=4096
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536,PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=SEG_PX=2048,PIPE_STREAMS=2" REPS=2 TAG=r5/piperestir4/ab BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_env.sh || exit 1
echo done
