# wave issue priority (s_setprio, variant builds): trace waves at 1 (libptx_p1.so) or the
# logic kernels' waves at 1 (libptx_p2.so) vs HEAD, same box
set -o pipefail
LIBS="libptx.so libptx_p1.so libptx_p2.so" REPS=3 TAG=prio_reuse BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_p1.so libptx_p2.so" REPS=1 TAG=prio_furn BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_p1.so libptx_p2.so" REPS=1 TAG=prio_gi BENCH_ARGS="--no-configs3 --workload gi" bash tools/ab_libs.sh || exit 1
