# round 5: the restructured hybrid-shift build: reuse / parity / node GPU tests, then benches vs
# the pre-hybrid kernels (libptx_pre.so) and JOB_STEP_WAVES=4 (libptx_js4.so)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_bands.py tests/test_node_engine.py tests/test_gpu_loopback.py -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/r5hyb2_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r5hyb2_tests.log; exit 1; }
tail -1 gpurun_out/r5hyb2_tests.log
VARIANTS="pre js4" SKIP_TESTS=1 REPS=2 TAG=r5hyb2 bash tools/cl/r5_multi_ab.sh
