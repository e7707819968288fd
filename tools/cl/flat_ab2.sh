# flattened instance loop from 3 instances: GPU suite; A/B of the threshold (FLAT_MIN_INST=1 / 1000) on C1 and C3
set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/flat2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/flat2_tests.log; exit 1; }
tail -1 gpurun_out/flat2_tests.log
AB=$'PTX_AB=\nPTX_AB=FLAT_MIN_INST=1000' REPS=2 TAG=ab_flat2 bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=FLAT_MIN_INST=1' REPS=1 TAG=ab_flat2_m BENCH_ARGS="--workload mcpt" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=FLAT_MIN_INST=1' REPS=1 TAG=ab_flat2_r BENCH_ARGS="--workload restir" bash tools/ab_env.sh || exit 1
grep -h '^{' gpurun_out/ab_flat2/run_1.log gpurun_out/ab_flat2/run_2.log | python -c 'import json,sys; [print(json.loads(l)["configs3_one_gpu"]["value"]) for l in sys.stdin]'
