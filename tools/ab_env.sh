#!/usr/bin/env bash
# A/B of environment knobs on one box: for each "VAR=val ..." line of $AB (newline-separated),
# one bench run (BENCH_ARGS) -> value per line.  usage: AB=$'PTX_AB=TRACE_SPLIT=1\nPTX_AB=TRACE_SPLIT=2' bash tools/ab_env.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
i=0
for rep in $(seq 1 ${REPS:-1}); do
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  env $line timeout -k 10 200 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/run_$i.log" 2>&1 || { echo "[$line] failed rc=$?"; tail -n 5 "$OUT/run_$i.log"; exit 1; }
  v=$(grep '^{' "$OUT/run_$i.log" | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')
  echo "rep $rep [$line] value ms frac: $v"
done <<< "$AB"
done
