# Q_SHADE shift-job hits: GPU suite, then same-box A/B vs the hit-compact build
set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/shade_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/shade_tests.log; exit 1; }
tail -1 gpurun_out/shade_tests.log
LIBS="libptx.so libptx_noshade.so" REPS=3 TAG=ab_shade bash tools/ab_libs.sh || exit 1
