# round-3 evidence at the final kernels: rocprofv3 stats + PMC + bench line per workload, then
# configs[3]'s 8 bands each timed alone with three measured re-cuts
set -o pipefail
ROUND=r3 WORKLOADS="${WLS:-reuse gi restir mcpt}" bash tools/round_evidence.sh || exit 1
timeout -k 10 600 python -u tools/band_alone.py --world 8 --recut 3 > gpurun_out/ev_recut.log 2>&1 || { echo "recut failed"; tail -5 gpurun_out/ev_recut.log; exit 1; }
tail -n 1 gpurun_out/ev_recut.log | cut -c1-300
