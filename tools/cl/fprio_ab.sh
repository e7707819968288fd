# the front (G-buffer + PT_1) of a pipelined frame on a high-priority stream (PTX_AB=FRONT_PRIO):
# quick parity, then same-box A/B (3 reps) on the headline
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/prio_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/prio_tests.log; exit 1; }
tail -1 gpurun_out/prio_tests.log
AB=$'PTX_AB=\nPTX_AB=FRONT_PRIO=1' REPS=3 TAG=ab_fprio BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
