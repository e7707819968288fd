# round 5: GI's launch-timed region in the production kernel mode (dynamic batches, as its
# pipelined frames now run): bench line + GI GPU tests
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_gi.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gitimed_tests.log 2>&1 || { echo "GI tests failed"; tail -30 gpurun_out/gitimed_tests.log; exit 1; }
tail -1 gpurun_out/gitimed_tests.log
LIBS="libptx.so" REPS=2 TAG=r5/gitimed BENCH_ARGS="--no-configs3 --workload gi" bash tools/ab_libs.sh || exit 1
