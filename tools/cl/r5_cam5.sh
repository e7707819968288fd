# round 5 (last): the headline's segments below 1024 px (static slots, 2 front sequences), still and moving
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=SEG_PX=768
PTX_LIB_PATH=$L PTX_AB=SEG_PX=512" REPS=2 TAG=r5/cam5/cam BENCH_ARGS="--no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=SEG_PX=768
PTX_LIB_PATH=$L PTX_AB=SEG_PX=512" REPS=2 TAG=r5/cam5/still BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
echo done
