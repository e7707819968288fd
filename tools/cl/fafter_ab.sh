# the next frame's front held until this frame's spatial sequences pass logic round r
# (PTX_AB=FRONT_AFTER=r): quick parity, then same-box A/B (2 reps) for r = 0 / 1 / 2
set -o pipefail
PTX_AB=FRONT_AFTER=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fafter_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fafter_tests.log; exit 1; }
tail -1 gpurun_out/fafter_tests.log
AB=$'PTX_AB=\nPTX_AB=FRONT_AFTER=0\nPTX_AB=FRONT_AFTER=1\nPTX_AB=FRONT_AFTER=2' REPS=2 TAG=ab_fafter BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
