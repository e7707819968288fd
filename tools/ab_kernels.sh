#!/usr/bin/env bash
# Per-kernel A/B: rocprofv3 --kernel-trace --stats of a short single-sequence bench per library
# (PTX_AB=PIPELINE_FRAMES=0: kernels do not share the chip with a second frame), then the
# average duration of every kernel side by side (static trace slots, the production mode since late
# round 5; EXTRA_AB=TRACE_DYN=1 for the dynamic batches).  usage: LIBS="libptx_a.so libptx.so" bash tools/ab_kernels.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
P=$R/pathtracerdemo_amd
TAG=${TAG:-abk}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for L in $LIBS; do
  PTX_LIB_PATH=$P/$L PTX_AB=PIPELINE_FRAMES=0${EXTRA_AB:+,$EXTRA_AB} timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$L" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$L.log" 2>&1 || { echo "$L rc=$?"; tail -5 "$OUT/$L.log"; exit 1; }
done
python3 - "$OUT" $LIBS <<'PY'
import csv, glob, sys
out, libs = sys.argv[1], sys.argv[2:]
tab = {}
for L in libs:
    f = glob.glob(f"{out}/{L}/**/run_kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        n = r["Name"].split("(")[0].replace("void ", "").replace("ptx::", "")
        tab.setdefault(n, {})[L] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6)
print(f"{'kernel':52s}" + "".join(f"{L[:22]:>24s}" for L in libs) + "   (avg us, total ms)")
for n, d in sorted(tab.items(), key=lambda kv: -max(v[2] for v in kv[1].values())):
    print(f"{n[:52]:52s}" + "".join(f"{d[L][0]:12.1f}{d[L][2]:12.2f}" if L in d else f"{'-':>24s}" for L in libs))
PY
