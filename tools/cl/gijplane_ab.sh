# GI spatial jobs in slot planes (PTX_AB=GI_JOB_PLANES=0: pixel-major): GI GPU tests, then A/B
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_gi.py tests/test_gpu_bands.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gijp_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gijp_tests.log; exit 1; }
tail -1 gpurun_out/gijp_tests.log
AB=$'PTX_AB=\nPTX_AB=GI_JOB_PLANES=0' REPS=3 TAG=ab_gijp BENCH_ARGS="--no-configs3 --workload gi" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=GI_JOB_PLANES=0' REPS=1 TAG=ab_gijp_f BENCH_ARGS="--no-configs3 --workload gi --scene c3_furnished" bash tools/ab_env.sh || exit 1
