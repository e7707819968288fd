# round 4: the motion temporal pass on the GPU (reuse suite incl. the moving-camera path), then
# the trace-tail breakdown by Visibility segments (diagnostic build)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_reuse.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_motion_tests.log 2>&1 \
    || { echo "reuse GPU tests failed"; tail -40 gpurun_out/r4_motion_tests.log; exit 1; }
tail -3 gpurun_out/r4_motion_tests.log
PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so timeout -k 10 300 python -u tools/trace_tail.py --frames 2 --out gpurun_out/r4_trace_tail3.json > gpurun_out/r4_trace_tail3.txt 2>&1 || { echo "tail failed"; tail -20 gpurun_out/r4_trace_tail3.txt; exit 1; }
tail -12 gpurun_out/r4_trace_tail3.txt
