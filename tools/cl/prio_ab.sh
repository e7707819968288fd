# a pipelined frame's back half on high-priority streams (PTX_AB=BACK_PRIO): quick parity, then
# same-box A/B (3 reps) on the headline, with 2 and 3 back sequences
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/prio_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/prio_tests.log; exit 1; }
tail -1 gpurun_out/prio_tests.log
AB=$'PTX_AB=\nPTX_AB=BACK_PRIO=1\nPTX_AB=BACK_PRIO=1,PIPE_BACK_STREAMS=3' REPS=3 TAG=ab_prio BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
