# round-2 session-5 evidence at HEAD: GPU suite + smoke, then every workload's rocprof / PMC /
# bench line (tools/r2_evidence.sh).  Then, here: ROUND=r2 bash tools/collect_profiles.sh
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_gpu_tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -30 gpurun_out/r2_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r2_smoke.log; exit 1; }
echo "smoke ok"
ROUND=r2 bash tools/r2_evidence.sh
