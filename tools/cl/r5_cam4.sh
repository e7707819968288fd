# round 5 (late): the headline's whole-image segment size, still and moving (static slots, 2 front sequences)
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=SEG_PX=1024
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1280
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1792" REPS=2 TAG=r5/cam4/cam BENCH_ARGS="--no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB=SEG_PX=1024
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1280
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1792" REPS=2 TAG=r5/cam4/still BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
echo done
