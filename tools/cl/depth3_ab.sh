# three frames in flight (PTX_AB=PIPE_DEPTH=3: a third frame context, round robin): GPU suite
# under depth 3 and under the default, then same-box A/B on the headline (3 reps), 4K and furnished
set -o pipefail
PTX_AB=PIPE_DEPTH=3 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/depth3_tests.log 2>&1 || { echo "depth-3 tests failed"; tail -30 gpurun_out/depth3_tests.log; exit 1; }
tail -1 gpurun_out/depth3_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/depth2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/depth2_tests.log; exit 1; }
tail -1 gpurun_out/depth2_tests.log
AB=$'PTX_AB=\nPTX_AB=PIPE_DEPTH=3' REPS=3 TAG=ab_depth3 BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=PIPE_DEPTH=3' REPS=1 TAG=ab_depth3_4k BENCH_ARGS="--no-configs3 --frame 3840x2160" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=PIPE_DEPTH=3' REPS=1 TAG=ab_depth3_f BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
