# GPU suite + smoke at the current default build
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -40 gpurun_out/r4_suite.log; exit 1; }
tail -1 gpurun_out/r4_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
