#!/usr/bin/env bash
# Kernel trace of the production (multi-stream) frame for a concurrency timeline
# (python tools/timeline.py gpurun_out/<tag>/trace/.../run_kernel_trace.csv).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-timeline}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
tail -c 600 "$OUT/bench.log"
