# round 4: root pre-filter dealt over the wave (PTX_ROOT_DEAL) on top of the Visibility restart
# pools -- GPU suite bit-exact, then same-box A/B of the headline: default build vs the
# PTX_ROOT_DEAL=0 build (libptx_alt.so) vs pools off (PTX_AB=RESTART_POOL=0), then launch tails
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_deal_tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -40 gpurun_out/r4_deal_tests.log; exit 1; }
tail -1 gpurun_out/r4_deal_tests.log
ALT=$PWD/pathtracerdemo_amd/libptx_alt.so
for rep in 1 2; do
  for v in deal nodeal nopool; do
    case $v in
      deal) env_ab=""; lib="";;
      nodeal) env_ab=""; lib=$ALT;;
      nopool) env_ab="RESTART_POOL=0"; lib="";;
    esac
    PTX_AB=$env_ab PTX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs3 > gpurun_out/r4_deal_$v.$rep.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4_deal_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])" gpurun_out/r4_deal_$v.$rep.log $v
  done
done
PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so timeout -k 10 300 python -u tools/trace_tail.py --frames 2 --out gpurun_out/r4_trace_tail5.json > gpurun_out/r4_trace_tail5.txt 2>&1 || { echo "tail failed"; tail -20 gpurun_out/r4_trace_tail5.txt; exit 1; }
head -20 gpurun_out/r4_trace_tail5.txt
