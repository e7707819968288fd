# compact fresh shift-job state: GPU suite, A/B vs the 96-byte layout; trace occupancy / segment A/B
set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fresh_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fresh_tests.log; exit 1; }
tail -1 gpurun_out/fresh_tests.log
LIBS="libptx.so libptx_nofresh.so" REPS=2 TAG=ab_fresh bash tools/ab_libs.sh || exit 1
bash tools/cl/occ_ab.sh
