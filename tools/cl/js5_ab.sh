# wjob_step alone at 5 waves per SIMD (-DJOB_STEP_WAVES=5) vs all logic kernels at 5 vs 4 (reuse)
set -o pipefail
LIBS="libptx.so libptx_js5.so libptx_lw5.so" REPS=3 TAG=ab_js5 BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
