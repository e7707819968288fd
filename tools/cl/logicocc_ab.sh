# logic-kernel occupancy re-checked with the 5-wave flattened trace: spatial start at 4 waves
# (-DSPATIAL_START_WAVES=4), start/step kernels at 5 (-DLOGIC_WAVES=5), against the default
set -o pipefail
LIBS="libptx.so libptx_ss4.so libptx_lw5.so" REPS=2 TAG=ab_logicocc BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
