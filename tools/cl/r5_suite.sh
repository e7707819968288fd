# round 5: GPU suite + smoke + the default bench line at the current build
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 300 --timeout-method thread > gpurun_out/r5/suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -60 gpurun_out/r5/suite.log; exit 1; }
tail -1 gpurun_out/r5/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 gpurun_out/r5/smoke.log; exit 1; }
tail -1 gpurun_out/r5/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r5/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r5/bench.log; exit 1; }
tail -1 gpurun_out/r5/bench.log | cut -c1-400
