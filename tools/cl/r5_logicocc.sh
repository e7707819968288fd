# round 5: the spatial pass's logic kernels' occupancy (wspatial_start 2 / 3 / 4 waves per SIMD,
# wjob_step 3 / 4 / 5) on the headline, same box
set -o pipefail
LIBS="libptx.so libptx_s2.so libptx_s4.so libptx_j3.so libptx_j5.so" REPS=2 TAG=r5/logicocc BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
