# round 5: pipelined TEST_MCPT frames on static trace slots -- segment size x sequences per context
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536,TRACE_DYN=0
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1280,TRACE_DYN=0
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1792,TRACE_DYN=0
PTX_LIB_PATH=$L PTX_AB=SEG_PX=2048,TRACE_DYN=0
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1792,TRACE_DYN=0,PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1024,TRACE_DYN=0,PIPE_STREAMS=2" REPS=2 TAG=r5/pipemcpt2/ab BENCH_ARGS="--workload mcpt --no-configs3" bash tools/ab_env.sh || exit 1
echo done
