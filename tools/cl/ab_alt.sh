# Same-box A/B of the default build against libptx_alt.so (make alt ALT_DEFS=...) on the
# headline (bench.py --no-cpu-baseline --no-configs3), REPS interleaved repetitions.
# usage: REPS=2 TAG=name bash tools/cl/ab_alt.sh
set -o pipefail
P=$PWD/pathtracerdemo_amd
TAG=${TAG:-ab}
for rep in $(seq 1 ${REPS:-2}); do
  for v in cur alt; do
    lib=""; [ "$v" = alt ] && lib=$P/libptx_alt.so
    PTX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs3 ${BENCH_ARGS:-} > gpurun_out/${TAG}_$v.$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/${TAG}_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])" gpurun_out/${TAG}_$v.$rep.log $v
  done
done
