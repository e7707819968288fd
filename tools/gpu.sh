#!/usr/bin/env bash
# One parametrised driver for the GPU-box steps (run under gpurun from the repo root):
#   bash tools/gpu.sh <step> <out-dir> [args...]
# Every step writes under gpurun_out/<out-dir>/, runs under its own time limit and exits non-zero
# on the first failure (the caller chains steps with &&, so nothing runs on the GPU after a fault).
#
#   suite   OUT [pytest args]   the GPU test suite (-m gpu), log in OUT/suite.log
#   smoke   OUT                 __graft_entry__.smoke()
#   bench   OUT NAME [bench.py args]   one bench line -> OUT/NAME.json (+ NAME.log)
#   profile OUT [bench.py args] rocprofv3 --kernel-trace --stats of `bench.py --profile-region` on the
#                               SHIPPED libptx.so (one launch sequence, one frame in flight: the
#                               region the line's event timing measures), then separate --pmc passes:
#                               FETCH_SIZE, WRITE_SIZE (HBM) and TCC_REQ/HIT/MISS (L2), and the same
#                               L2 pass over a streaming copy of known bytes (tools/l2_calib.py)
#   bands   OUT NAME [band_alone.py args]  configs[3]'s bands, each alone (tools/band_alone.py) ->
#                               OUT/NAME.jsonl; PROXY_US (default 110) sets the exchange stand-in,
#                               EXTRA_AB more PTX_AB switches (with PTX_LIB_PATH=.../libptx_ab.so)
#   simd    OUT WORKLOAD        lane use per traversal region (tools/simd_util.py; measurement build)
#   kstats  OUT [bench.py args] kernel trace + stats of the profile region (PTX_LIB_PATH honoured)
#   sq      OUT [bench.py args] one --pmc pass of SQ wave-cycle / instruction counters (profile region)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
step=$1
O=gpurun_out/$2
shift 2
mkdir -p "$O"
case "$step" in
suite)
    timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread "$@" > "$O/suite.log" 2>&1 \
        || { echo "GPU suite failed"; tail -40 "$O/suite.log"; exit 1; }
    tail -1 "$O/suite.log" ;;
smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
    tail -1 "$O/smoke.log" ;;
bench)
    name=$1
    shift
    timeout -k 10 600 python -u bench.py "$@" > "$O/$name.log" 2>&1 || { echo "bench $name failed"; tail -20 "$O/$name.log"; exit 1; }
    grep '^{' "$O/$name.log" | tail -n 1 > "$O/$name.json"
    python3 - "$O/$name.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
rf = d.get("roofline", {})
c3 = d.get("configs3_one_gpu") or {}
print(sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "frac", rf.get("frac"), "frac+qio", rf.get("frac_with_queue_io"),
      "launch_ms", rf.get("avg_launch_ms"), "4k", c3.get("value"), "parity", (d.get("parity") or {}).get("bit_exact"),
      "clips", (d.get("motion_clip_px") or {}).get("pixels"), "lib", d.get("library", {}).get("build"))
EOF
    ;;
profile)
    cd /tmp && export TMPDIR=/tmp
    P="$R/$O"
    unset PTX_AB PTX_LIB_PATH
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- \
        python3 "$R/bench.py" --profile-region --steps 20 --warmup 3 "$@" > "$P/bench_trace.log" 2>&1 \
        || { echo "trace rc=$?"; tail -5 "$P/bench_trace.log"; exit 1; }
    grep '^{' "$P/bench_trace.log" | tail -n 1 > "$P/bench_line_profile_region.json"
    echo "trace ok"
    for C in FETCH_SIZE WRITE_SIZE "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
        tag=$(echo "$C" | cut -d' ' -f1)
        timeout -s KILL 120 rocprofv3 --pmc $C -d "$P/pmc_$tag" -o run --output-format csv -- \
            python3 "$R/bench.py" --profile-region --steps 5 --warmup 1 "$@" > "$P/bench_$tag.log" 2>&1 \
            || { echo "pmc $tag rc=$?"; tail -5 "$P/bench_$tag.log"; exit 1; }
        echo "pmc $tag ok"
    done
    timeout -s KILL 120 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum -d "$P/pmc_calib" -o run --output-format csv -- \
        python3 "$R/tools/l2_calib.py" > "$P/l2_calib.log" 2>&1 || { echo "l2 calib rc=$?"; tail -5 "$P/l2_calib.log"; exit 1; }
    echo "l2 calib ok" ;;
kstats)  # rocprofv3 --kernel-trace --stats of the profile region only, on the library PTX_LIB_PATH names
         # (default: the shipped one) -> OUT/trace/; tools/kstats.py prints per-kernel averages
    cd /tmp && export TMPDIR=/tmp
    P="$R/$O"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- \
        python3 "$R/bench.py" --profile-region --steps 20 --warmup 3 "$@" > "$P/bench_trace.log" 2>&1 \
        || { echo "kstats rc=$?"; tail -5 "$P/bench_trace.log"; exit 1; }
    python3 "$R/tools/kstats.py" "$P/trace/run_kernel_stats.csv" ;;
sq)  # one --pmc pass of 8 SQ counters over the profile region (wave cycles: parked / issue-stalled /
     # issuing; instruction mix) -> OUT/pmc_sq/; tools/sq_table.py summarises it per kernel
    cd /tmp && export TMPDIR=/tmp
    P="$R/$O"
    unset PTX_AB PTX_LIB_PATH
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d "$P/pmc_sq" -o run --output-format csv -- \
        python3 "$R/bench.py" --profile-region --steps 5 --warmup 1 "$@" > "$P/bench_sq.log" 2>&1 \
        || { echo "pmc sq rc=$?"; tail -5 "$P/bench_sq.log"; exit 1; }
    echo "pmc sq ok" ;;
bands)
    name=$1
    shift
    PTX_AB=HALO_PROXY_US=${PROXY_US:-110}${EXTRA_AB:+,$EXTRA_AB} timeout -k 10 900 python -u tools/band_alone.py "$@" > "$O/$name.jsonl" 2> "$O/$name.err" \
        || { echo "bands $name failed"; tail -5 "$O/$name.err"; exit 1; }
    cut -c1-400 "$O/$name.jsonl" ;;
simd)
    timeout -k 10 300 python -u tools/simd_util.py --workload "$1" > "$O/simd_$1.txt" 2>&1 || { echo "simd failed"; tail -5 "$O/simd_$1.txt"; exit 1; }
    tail -8 "$O/simd_$1.txt" ;;
*)
    echo "unknown step $step"; exit 2 ;;
esac
