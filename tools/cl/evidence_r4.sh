# round-4 evidence at the final kernels: rocprofv3 stats + PMC (FETCH_SIZE, WRITE_SIZE) + the
# bench line per workload (WLS, default the headline reuse + GI; restir mcpt in a second call)
set -o pipefail
ROUND=r4 WORKLOADS="${WLS:-reuse gi}" bash tools/round_evidence.sh || exit 1
