set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/uni_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/uni_tests.log; exit 1; }
tail -1 gpurun_out/uni_tests.log
LIBS="libptx.so libptx_uni0.so" REPS=2 TAG=ab_uni bash tools/ab_libs.sh
