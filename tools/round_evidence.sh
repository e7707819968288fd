#!/usr/bin/env bash
# Round evidence for profiles/<round>/<workload>/: rocprofv3 kernel trace + stats, the two
# PMC passes (FETCH_SIZE, WRITE_SIZE) and the bench line (with its CPU baseline) of the
# same build.  usage: ROUND=r1 WORKLOADS="reuse restir mcpt" bash tools/round_evidence.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
ROUND=${ROUND:-r1}
for WL in ${WORKLOADS:-reuse restir mcpt}; do
  # (every whole-image pipeline runs static trace slots since late round 5, as the profile's
  # one-frame-in-flight region does: no TRACE_DYN override)
  TAG=${ROUND}_$WL BENCH_ARGS="--workload $WL" bash tools/profile.sh || { echo "profile $WL failed"; exit 1; }
  timeout -k 10 400 python3 bench.py --workload "$WL" --steps 20 --warmup 3 > "gpurun_out/bench_${ROUND}_$WL.log" 2>&1 \
    || { echo "bench $WL failed"; exit 1; }
  echo "$WL: $(tail -n 1 gpurun_out/bench_${ROUND}_$WL.log | cut -c1-200)"
done
