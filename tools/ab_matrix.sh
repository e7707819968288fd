#!/usr/bin/env bash
# A/B matrix: for each bench argument set in $ARGSETS (newline-separated) and each env line in
# $AB, one bench run.  usage: ARGSETS=$'--workload gi\n--workload mcpt' AB=$'X=0\nX=1' bash tools/ab_matrix.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT=gpurun_out/${TAG:-abm}
mkdir -p "$OUT"
i=0
while IFS= read -r args; do
  while IFS= read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    env $line timeout -k 10 240 python3 bench.py --steps ${STEPS:-15} --warmup 4 --no-cpu-baseline $args > "$OUT/run_$i.log" 2>&1 || { echo "[$args | $line] failed rc=$?"; tail -n 5 "$OUT/run_$i.log"; exit 1; }
    v=$(grep '^{' "$OUT/run_$i.log" | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')
    echo "[$args | $line] value ms frac: $v"
  done <<< "$AB"
done <<< "$ARGSETS"
