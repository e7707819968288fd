# round 5 (last): the headline at 1024-px static slots -- front / back sequences per context, still and moving
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=1
PTX_LIB_PATH=$L PTX_AB=PIPE_BACK_STREAMS=1
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=3" REPS=2 TAG=r5/cam6/cam BENCH_ARGS="--no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=1
PTX_LIB_PATH=$L PTX_AB=PIPE_BACK_STREAMS=1
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=3" REPS=2 TAG=r5/cam6/still BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
echo done
