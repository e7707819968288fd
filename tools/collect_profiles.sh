#!/usr/bin/env bash
# Copy one GPU call's rocprofv3 evidence from gpurun_out/ (scratch) into the tracked
# profiles/<round>/<workload>/ and refresh profiles/hbm_traffic.json + profiles/limiters.json.
#
# Round 6 layout (tools/gpu.sh): ROUND=r6 SRC=gpurun_out/r6/<case> bash tools/collect_profiles.sh
#   SRC/prof_<wl>/     tools/gpu.sh profile  (kernel trace + stats, PMC passes, L2 calibration)
#   SRC/<wl>.json      tools/gpu.sh bench    (the workload's bench line of the same build)
#   SRC/simd_<wl>.txt  tools/gpu.sh simd     (optional: lane use per traversal region)
# Rounds 1-5 (tools/round_evidence.sh): no SRC; reads gpurun_out/prof_<ROUND>_<wl>/.
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
ROUND=${ROUND:-r1}
declare -A SCENE=([reuse]=c3_interior_32 [gi]=c3_interior_32 [restir]=dummy_scene_1 [mcpt]=dummy_scene_1)
for WL in ${WORKLOADS:-reuse restir mcpt gi}; do
  if [ -n "${SRC:-}" ]; then src=$SRC/prof_$WL; line=$SRC/$WL.json; simd=$SRC/simd_$WL.txt
  else src=gpurun_out/prof_${ROUND}_$WL; line=gpurun_out/bench_${ROUND}_$WL.log; simd=; fi
  [ -d "$src" ] || { echo "skip $WL (no $src)"; continue; }
  dst=profiles/$ROUND/$WL
  mkdir -p "$dst"
  cp "$src/trace/run_kernel_stats.csv" "$dst/kernel_stats.csv"
  cp "$src/trace/run_kernel_trace.csv" "$dst/kernel_trace.csv"
  for p in "$src"/pmc_*; do
    mkdir -p "$dst/$(basename "$p")"
    cp "$p/run_counter_collection.csv" "$dst/$(basename "$p")/counter_collection.csv"
  done
  cp "$src/bench_trace.log" "$dst/bench_under_rocprof.log"
  [ -f "$src/bench_line_profile_region.json" ] && cp "$src/bench_line_profile_region.json" "$dst/"
  grep '^{' "$line" | tail -n 1 > "$dst/bench_line.json"
  [ -n "$simd" ] && [ -f "$simd" ] && cp "$simd" "$dst/simd_util.txt"
  # the timed roofline symbol only (GI: the closest-hit instance, not the any-hit one); the
  # flattened walk at 5 waves per SIMD runs every scene since round 5 (kFlatMinInstances = 1)
  KN="trace_queue<false, 5, false, true, false"
  KEY="$WL:${SCENE[$WL]}:trace_queue:1920x1080"
  if [ -d "$dst/pmc_TCC_REQ_sum" ]; then
    python3 tools/limiters.py "$dst" "$KEY" "$KN" $( [ -f "$dst/simd_util.txt" ] && echo "$dst/simd_util.txt" ) > /dev/null
  else
    python3 tools/hbm_traffic.py "$dst" "$KEY" "$KN" > /dev/null
  fi
  # the bench line carries the PMC traffic (and limiters) of THIS build's passes (the bench ran
  # before them and looked up the previous entries)
  python3 - "$dst" "$KEY" <<'PY'
import json, os, sys
d, key = sys.argv[1], sys.argv[2]
db = json.load(open("profiles/hbm_traffic.json"))
line = json.load(open(f"{d}/bench_line.json"))
rf = line["roofline"]
rf["traffic"] = db[key]["bytes_per_launch"]
rf["traffic_source"] = (f"{db[key]['source']}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of the same build, "
                        f"2*FETCH_SIZE + WRITE_SIZE per launch of {db[key].get('kernel', 'trace_queue')}")
lim = json.load(open("profiles/limiters.json")).get(key) if os.path.exists("profiles/limiters.json") else None
if lim:
    ms = rf["avg_launch_ms"] * 1e-3
    lim = dict(lim)
    if lim.get("l2_bytes_per_launch"):
        lim["l2_achieved_gbs"] = round(lim["l2_bytes_per_launch"] / ms / 1e9, 1)
        lim["l2_peak_gbs"] = 34500.0
        lim["l2_frac"] = round(lim["l2_bytes_per_launch"] / ms / 1e9 / 34500.0, 4)
    lim["hbm_traffic_frac"] = round(rf["traffic"] / ms / 1e9 / 8000.0, 4)
    rf["limiters"] = lim
json.dump(line, open(f"{d}/bench_line.json", "w"))
PY
  echo "$WL -> $dst"
done
