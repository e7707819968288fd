#!/usr/bin/env bash
# Copy a round_evidence.sh run's rocprofv3 summaries from gpurun_out/ (scratch) into the
# tracked profiles/<round>/<workload>/ and refresh profiles/hbm_traffic.json.
# usage: ROUND=r1 WORKLOADS="reuse restir mcpt gi" bash tools/collect_profiles.sh
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
ROUND=${ROUND:-r1}
declare -A SCENE=([reuse]=c3_interior_32 [gi]=c3_interior_32 [restir]=dummy_scene_1 [mcpt]=dummy_scene_1)
for WL in ${WORKLOADS:-reuse restir mcpt gi}; do
  src=gpurun_out/prof_${ROUND}_$WL
  dst=profiles/$ROUND/$WL
  mkdir -p "$dst/pmc_FETCH_SIZE" "$dst/pmc_WRITE_SIZE"
  cp "$src/trace/run_kernel_stats.csv" "$dst/kernel_stats.csv"
  cp "$src/trace/run_kernel_trace.csv" "$dst/kernel_trace.csv"
  cp "$src/pmc_FETCH_SIZE/run_counter_collection.csv" "$dst/pmc_FETCH_SIZE/counter_collection.csv"
  cp "$src/pmc_WRITE_SIZE/run_counter_collection.csv" "$dst/pmc_WRITE_SIZE/counter_collection.csv"
  cp "$src/bench_trace.log" "$dst/bench_under_rocprof.log"
  tail -n 1 "gpurun_out/bench_${ROUND}_$WL.log" > "$dst/bench_line.json"
  # the timed roofline symbol only (GI: the closest-hit instance, not the any-hit one); the
  # flattened walk at 5 waves per SIMD runs every scene since round 5 (kFlatMinInstances = 1)
  KN="trace_queue<false, 5, false, true, false"
  python3 tools/hbm_traffic.py "$dst" "$WL:${SCENE[$WL]}:trace_queue:1920x1080" "$KN" > /dev/null
  # the bench line carries the PMC traffic of THIS build's passes (the bench ran first and
  # looked up the previous entry)
  python3 - "$dst" "$WL:${SCENE[$WL]}:trace_queue:1920x1080" <<'PY'
import json, sys
d, key = sys.argv[1], sys.argv[2]
db = json.load(open("profiles/hbm_traffic.json"))
line = json.load(open(f"{d}/bench_line.json"))
line["roofline"]["traffic"] = db[key]["bytes_per_launch"]
line["roofline"]["traffic_source"] = f"{db[key]['source']}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of the same bench command, 2*FETCH_SIZE + WRITE_SIZE per launch of {db[key].get('kernel', 'trace_queue')}"
json.dump(line, open(f"{d}/bench_line.json", "w"))
PY
  echo "$WL -> $dst"
done
