# start/step kernels at 5 waves per SIMD (-DLOGIC_WAVES=5, libptx_lw5.so) vs 4, every workload
set -o pipefail
for wl in reuse gi restir mcpt; do
  LIBS="libptx.so libptx_lw5.so" REPS=2 TAG=ab_lw5_$wl BENCH_ARGS="--no-configs3 --workload $wl" bash tools/ab_libs.sh || exit 1
done
