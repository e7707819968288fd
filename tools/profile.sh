#!/usr/bin/env bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r1}
ARGS=${BENCH_ARGS:-}
cd /tmp && export TMPDIR=/tmp
# one launch sequence per pass: per-kernel durations then match bench.py's launch-timing
# region (PTX_FLAG_SINGLE_STREAM); the two-stream production overlap is measured by the
# bench's headline value, not by per-kernel averages
# and one frame in flight (frame pipelining overlaps consecutive frames' kernels); EXTRA_AB
# adds switches (e.g. TRACE_DYN=1: the dynamic trace batches, the reuse pipeline's default
# before late round 5)
export PTX_AB="WAVE_STREAMS=1,PIPELINE_FRAMES=0${EXTRA_AB:+,$EXTRA_AB}"
# (the shipped libptx.so compiles these switches to their defaults since round 5: the profile
# runs the measurement build of the same sources, make -C pathtracerdemo_amd/csrc ab)
export PTX_LIB_PATH="${PTX_LIB_PATH:-$R/pathtracerdemo_amd/libptx_ab.so}"
[ -f "$PTX_LIB_PATH" ] || { echo "missing $PTX_LIB_PATH (make -C pathtracerdemo_amd/csrc ab)"; exit 1; }
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-configs3 $ARGS > "$OUT/bench_trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
echo "trace ok"; tail -n 1 "$OUT/bench_trace.log"
if [ "${NO_PMC:-0}" = "1" ]; then exit 0; fi
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/pmc_$C" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-configs3 $ARGS > "$OUT/bench_$C.log" 2>&1 || { echo "pmc $C rc=$?"; exit 1; }
  echo "pmc $C ok"
done
