# Per-kernel A/B: rocprofv3 kernel stats of the headline bench with the default build and with
# libptx_alt.so (make alt ALT_DEFS=...), same box.  usage: TAG=name bash tools/cl/r5_kprof_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-kab}
for v in cur alt; do
  lib=""; [ "$v" = alt ] && lib=$R/pathtracerdemo_amd/libptx_alt.so
  mkdir -p $R/gpurun_out/$TAG/$v
  PTX_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/$v -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-configs3 --steps 10 --warmup 3 > $R/gpurun_out/$TAG/$v/bench.log 2>&1 \
    || { echo "prof $v failed"; tail -5 $R/gpurun_out/$TAG/$v/bench.log; exit 1; }
done
python3 - "$R/gpurun_out/$TAG" <<'EOF'
import csv, glob, sys
def load(v):
    f = glob.glob(f"{sys.argv[1]}/{v}/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"][:70]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f))}
a, b = load("cur"), load("alt")
for k in sorted(a, key=lambda k: -a[k][0] * a[k][1])[:16]:
    if k in b:
        print(f"{k:70s} {a[k][0]:5d} cur {a[k][1]:8.1f} alt {b[k][1]:8.1f} us  {a[k][1] / b[k][1]:.3f}")
EOF
