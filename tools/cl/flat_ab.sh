# flattened instance loop: GPU suite, then same-box A/B (flat vs PTX_FLAT_INST=0) per workload
set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/flat_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/flat_tests.log; exit 1; }
tail -1 gpurun_out/flat_tests.log
LIBS="libptx.so libptx_noflat.so" REPS=2 TAG=ab_flat bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_noflat.so" REPS=1 TAG=ab_flat_f BENCH_ARGS="--scene c3_furnished" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_noflat.so" REPS=1 TAG=ab_flat_m BENCH_ARGS="--workload mcpt" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_noflat.so" REPS=1 TAG=ab_flat_g BENCH_ARGS="--workload gi" bash tools/ab_libs.sh || exit 1
for L in libptx.so libptx_noflat.so; do grep -h configs3 gpurun_out/ab_flat/*.log | head -0; done
