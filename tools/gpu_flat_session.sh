set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/flat_gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED rc=$?"; tail -20 gpurun_out/flat_gpu_tests.log; exit 1; }
tail -3 gpurun_out/flat_gpu_tests.log
AB=$'PTX_TRACE_OCC=4\nPTX_TRACE_OCC=5' REPS=2 TAG=occ_reuse bash tools/ab_env.sh || exit 1
BENCH_ARGS="--workload gi" AB=$'PTX_TRACE_OCC=4\nPTX_TRACE_OCC=5' REPS=2 TAG=occ_gi bash tools/ab_env.sh || exit 1
BENCH_ARGS="--workload mcpt" AB=$'PTX_TRACE_OCC=4\nPTX_TRACE_OCC=5' REPS=2 TAG=occ_mcpt bash tools/ab_env.sh || exit 1
BENCH_ARGS="--workload restir" AB=$'PTX_TRACE_OCC=4\nPTX_TRACE_OCC=5' REPS=2 TAG=occ_restir bash tools/ab_env.sh || exit 1
