# round 5: evidence at the streamed trace walk (reuse + GI): rocprof stats, PMC, bench lines
set -o pipefail
ROUND=r5 WORKLOADS="reuse gi" bash tools/round_evidence.sh || exit 1
