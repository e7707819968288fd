# round 5 (late): trace-launch switches at the static-slot pipelined shapes (headline reuse, C1 ReSTIR)
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
for wl in reuse restir; do
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=TRACE_SPLIT=2
PTX_LIB_PATH=$L PTX_AB=TRACE_OCC=4
PTX_LIB_PATH=$L PTX_AB=TRACE_OCC=6
PTX_LIB_PATH=$L PTX_AB=SEG_CLUSTER=4" REPS=2 TAG=r5/shape2/$wl BENCH_ARGS="--workload $wl --no-configs3" bash tools/ab_env.sh || exit 1
done
echo done
