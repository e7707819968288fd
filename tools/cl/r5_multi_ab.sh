# Same-box A/B of the default build against several variant builds (make -C pathtracerdemo_amd/csrc
# variant NAME=x ALT_DEFS=...): first the bit-exact GPU parity + reuse tests on every variant, then
# REPS interleaved headline benches (SKIP_TESTS=1: benches only).  usage: VARIANTS="e1 e2" REPS=2 TAG=name bash tools/cl/r5_multi_ab.sh
set -o pipefail
P=$PWD/pathtracerdemo_amd
TAG=${TAG:-mab}
for v in ${VARIANTS}; do
  [ -n "${SKIP_TESTS:-}" ] && break
  PTX_LIB_PATH=$P/libptx_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reuse.py -m gpu -x -q \
      --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests_$v.log 2>&1 \
    || { echo "tests $v failed"; tail -30 gpurun_out/${TAG}_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/${TAG}_tests_$v.log)"
done
for rep in $(seq 1 ${REPS:-2}); do
  for v in cur ${VARIANTS}; do
    lib=""; [ "$v" != cur ] && lib=$P/libptx_$v.so
    PTX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs3 ${BENCH_ARGS:-} > gpurun_out/${TAG}_$v.$rep.log 2>&1 \
      || { echo "bench $v failed"; tail -5 gpurun_out/${TAG}_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])" gpurun_out/${TAG}_$v.$rep.log $v
  done
done
