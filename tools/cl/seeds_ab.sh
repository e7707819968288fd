# fresh shift jobs keep rSeed[1] in their state and the neighbour summary carries the sample's
# seed words (32 B): no reservoir gather in wjob_step's fresh-job load or wspatial_start's forward
# jobs.  GPU reuse / bands suites, then same-box A/B against the previous build (libptx_base.so)
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_bands.py tests/test_gpu_debug_fill.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/seeds_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/seeds_tests.log; exit 1; }
tail -1 gpurun_out/seeds_tests.log
LIBS="libptx.so libptx_base.so" REPS=3 TAG=ab_seeds BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_base.so" REPS=1 TAG=ab_seeds_f BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_libs.sh || exit 1
