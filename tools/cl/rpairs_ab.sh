# root pre-filter two roots per iteration (-DPTX_ROOT_PAIRS=1, libptx_rp.so) vs HEAD:
# GPU parity of the variant first, then same-box bench A/B per workload
set -o pipefail
PARITY=1 PARITY_LIBS=libptx_rp.so PARITY_TESTS="tests/test_gpu_reuse.py tests/test_gpu_gi.py tests/test_gpu_cull.py" \
  LIBS="libptx.so libptx_rp.so" REPS=3 TAG=rp_reuse BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_rp.so" REPS=2 TAG=rp_furn BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_rp.so" REPS=1 TAG=rp_gi BENCH_ARGS="--no-configs3 --workload gi" bash tools/ab_libs.sh || exit 1
