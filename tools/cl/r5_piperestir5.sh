# round 5: pipelined ReSTIR frames -- segment size x sequences per context, second sweep
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=SEG_PX=2048,PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=SEG_PX=2048,PIPE_STREAMS=3
PTX_LIB_PATH=$L PTX_AB=SEG_PX=2560,PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1792,PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=SEG_PX=2048,PIPE_STREAMS=2,PIPE_DEPTH=3" REPS=2 TAG=r5/piperestir5/ab BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_env.sh || exit 1
echo done
