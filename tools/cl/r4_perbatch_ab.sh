# round 4: the per-batch dynamic trace loop restored as the default (PTX_RESTART_POOL=0):
# GPU suite, then same-box A/B: old = round-start build, cur = default, alt = PTX_RESTART_POOL=1
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pb_tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -40 gpurun_out/r4_pb_tests.log; exit 1; }
tail -1 gpurun_out/r4_pb_tests.log
P=$PWD/pathtracerdemo_amd
for rep in 1 2; do
  for v in old cur alt; do
    case $v in
      old) lib=$P/libptx_old.so;;
      cur) lib="";;
      alt) lib=$P/libptx_alt.so;;
    esac
    PTX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs3 > gpurun_out/r4_pb_$v.$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r4_pb_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])" gpurun_out/r4_pb_$v.$rep.log $v
  done
done
