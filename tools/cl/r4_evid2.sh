# round-4 evidence for the other workloads (GI, ReSTIR, TEST_MCPT) + smoke()
set -o pipefail
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
WLS="gi restir mcpt" bash tools/cl/evidence_r4.sh
