# round 5: segment size per pipeline at the streamed walk (reuse headline, GI, TEST_MCPT; 1080p)
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
for wl in reuse gi mcpt; do
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=SEG_PX=768
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536
PTX_LIB_PATH=$L PTX_AB=SEG_PX=2048" REPS=2 TAG=r5/segall/$wl BENCH_ARGS="--workload $wl --no-configs3" bash tools/ab_env.sh || exit 1
done
echo done
