# dynamic trace batches with the tail of every head's chunk dealt as 16-query quarters
# (PTX_AB=TAIL_SPLIT=S: the last S batches of each chunk): parity under S = 512, then A/B
set -o pipefail
PTX_AB=TAIL_SPLIT=512 timeout -k 10 500 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_gi.py tests/test_gpu_bands.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tail_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tail_tests.log; exit 1; }
tail -1 gpurun_out/tail_tests.log
AB=$'PTX_AB=\nPTX_AB=TAIL_SPLIT=128\nPTX_AB=TAIL_SPLIT=512\nPTX_AB=TAIL_SPLIT=2048'
AB="$AB" REPS=2 TAG=ab_tail BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
AB="$AB" REPS=1 TAG=ab_tail_gi BENCH_ARGS="--no-configs3 --workload gi" bash tools/ab_env.sh || exit 1
