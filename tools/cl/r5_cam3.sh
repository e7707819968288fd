# round 5 (late): the moving headline camera -- back-half sequences and segment size at the static shape
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=PIPE_BACK_STREAMS=1
PTX_LIB_PATH=$L PTX_AB=PIPE_BACK_STREAMS=3
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1024
PTX_LIB_PATH=$L PTX_AB=SEG_PX=2560" REPS=2 TAG=r5/cam3 BENCH_ARGS="--no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
echo done
