# the segment split between a pipelined frame's two back sequences (PTX_AB=BACK_SPLIT=<percent of
# the first>; the wave timeline showed the second sequence ~0.5 ms behind the first): quick
# parity at 60, then same-box A/B (2 reps) at 50 / 55 / 60 / 65
set -o pipefail
PTX_AB=BACK_SPLIT=60 timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bsplit_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/bsplit_tests.log; exit 1; }
tail -1 gpurun_out/bsplit_tests.log
AB=$'PTX_AB=\nPTX_AB=BACK_SPLIT=55\nPTX_AB=BACK_SPLIT=60\nPTX_AB=BACK_SPLIT=65' REPS=2 TAG=ab_bsplit BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
