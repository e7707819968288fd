# round 4: Visibility restart pools (trace_lanes) -- GPU suite bit-exact, then same-box A/B of the
# headline with the pools on / off (PTX_AB=RESTART_POOL=0), then the launch tails with pools
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pool_tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -40 gpurun_out/r4_pool_tests.log; exit 1; }
tail -1 gpurun_out/r4_pool_tests.log
for rep in 1 2; do
  for ab in RESTART_POOL=1 RESTART_POOL=0; do
    PTX_AB=$ab timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs3 > gpurun_out/r4_pool_$ab.$rep.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4_pool_$ab.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])" gpurun_out/r4_pool_$ab.$rep.log $ab
  done
done
PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so timeout -k 10 300 python -u tools/trace_tail.py --frames 2 --out gpurun_out/r4_trace_tail4.json > gpurun_out/r4_trace_tail4.txt 2>&1 || { echo "tail failed"; tail -20 gpurun_out/r4_trace_tail4.txt; exit 1; }
head -20 gpurun_out/r4_trace_tail4.txt
