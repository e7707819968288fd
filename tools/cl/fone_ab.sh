# the reuse pipeline's PT_4 as one launch, replays traced inline (wfinal_one): GPU suite, then
# same-box A/B against PTX_AB=FINAL_ONE=0 (the queued 7-launch chain) on the headline (3 reps)
# and the furnished scene
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fone_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fone_tests.log; exit 1; }
tail -1 gpurun_out/fone_tests.log
AB=$'PTX_AB=\nPTX_AB=FINAL_ONE=0' REPS=3 TAG=ab_fone BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=FINAL_ONE=0' REPS=1 TAG=ab_fone_f BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
