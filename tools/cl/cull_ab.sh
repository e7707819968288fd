# instance cull: GPU suite, then same-box A/B (cull vs PTX_INST_CULL=0 build) on C3 and the furnished C3
set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cull_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/cull_tests.log; exit 1; }
tail -1 gpurun_out/cull_tests.log
LIBS="libptx.so libptx_nocull.so" REPS=2 TAG=ab_cull bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_nocull.so" REPS=1 TAG=ab_cull_f BENCH_ARGS="--scene c3_furnished" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_nocull.so" REPS=1 TAG=ab_cull_m BENCH_ARGS="--workload mcpt" bash tools/ab_libs.sh || exit 1
