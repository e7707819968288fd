# what the driver runs at round end, on one GPU: the GPU suite, smoke(), the default bench line
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -30 gpurun_out/final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/final_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/final_bench.log; exit 1; }
grep '^{' gpurun_out/final_bench.log | tail -n 1 | cut -c1-400
