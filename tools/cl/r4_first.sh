# round 4, first box: GPU suite + the default bench line (new parity / cores fields) + the
# trace-launch tail analysis of the launch-timed region (diagnostic build, tools/trace_tail.py)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -30 gpurun_out/r4_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4_gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4_bench.log; exit 1; }
grep '^{' gpurun_out/r4_bench.log | tail -n 1 | cut -c1-300
PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so timeout -k 10 300 python -u tools/trace_tail.py --out gpurun_out/r4_trace_tail.json > gpurun_out/r4_trace_tail.txt 2>&1 || { echo "tail failed"; tail -20 gpurun_out/r4_trace_tail.txt; exit 1; }
cat gpurun_out/r4_trace_tail.txt
