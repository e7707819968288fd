# round 5 (late): the moving GI camera at the static-slot shape vs one front sequence / dynamic batches
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=1
PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=1
PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=1,PIPE_STREAMS=1" REPS=2 TAG=r5/gicam2 BENCH_ARGS="--workload gi --no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=1" REPS=2 TAG=r5/cam2 BENCH_ARGS="--no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
echo done
