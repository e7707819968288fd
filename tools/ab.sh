#!/usr/bin/env bash
# A/B bench runs on one box: each line of $AB_FILE (or AB env, ';'-separated) is
# "<label>|<env assignments>|<bench args>".  Prints the bench JSON line per config.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/ab
IFS=';' read -ra CFGS <<< "${AB:-base||}"
for c in "${CFGS[@]}"; do
  IFS='|' read -r label envs args <<< "$c"
  env $envs timeout -k 10 ${AB_TIMEOUT:-240} python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline $args \
      > "gpurun_out/ab/$label.log" 2>&1 || { echo "$label rc=$?"; tail -5 "gpurun_out/ab/$label.log"; exit 1; }
  echo "$label: $(tail -n 1 gpurun_out/ab/$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["kernel_ms"])')"
done
