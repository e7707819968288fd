# round 4: band motion halo tests first, then the whole GPU suite, the LDS-transmission A/B,
# the bench line, the moving-camera line and the headline's rocprof / PMC evidence
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_bands.py -x -v --timeout 240 --timeout-method thread -k "moving or motion or communicator" > gpurun_out/r4_bandmotion_tests.log 2>&1 \
    || { echo "band motion tests failed"; tail -40 gpurun_out/r4_bandmotion_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r4_bandmotion_tests.log | tail -6
bash tools/cl/r4_mid3.sh
