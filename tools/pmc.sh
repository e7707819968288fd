#!/usr/bin/env bash
# PMC counter passes on a short bench run (one rocprofv3 invocation per counter group).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-pmc}
ARGS=${BENCH_ARGS:-}
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
if [ "${LIST:-0}" = "1" ]; then timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1; echo "list rc=$?"; fi
i=0
for G in ${GROUPS_:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"}; do :; done
while IFS= read -r G; do
  [ -z "$G" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $G -d "$OUT/g$i" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline $ARGS > "$OUT/g$i.log" 2>&1 || { echo "group $i rc=$?"; exit 1; }
  echo "group $i ok: $G"
done < "${GROUPS_FILE:-$R/tools/pmc_groups.txt}"
