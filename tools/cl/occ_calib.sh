# SQ occupancy calibration (tools/cl/occ_calib.hip) and the same counters on the reuse bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/occ"; mkdir -p "$OUT"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/calib" -o run --output-format csv -- "$R/tools/cl/occ_calib" > "$OUT/calib.log" 2>&1 || { echo "calib rc=$?"; exit 1; }
echo calib ok
export PTX_AB="WAVE_STREAMS=1,PIPELINE_FRAMES=0,TRACE_DYN=1"
timeout -s KILL 200 rocprofv3 --pmc $C -d "$OUT/bench" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; exit 1; }
echo bench ok
