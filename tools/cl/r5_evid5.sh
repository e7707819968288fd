# round 5 (late): evidence at the pipelined static-slot launch shapes -- rocprof stats, PMC, bench
# lines of all four workloads
set -o pipefail
ROUND=r5 WORKLOADS="reuse gi restir mcpt" bash tools/round_evidence.sh || exit 1
