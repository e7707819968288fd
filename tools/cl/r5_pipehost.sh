# round 5 (late): pipelined ReSTIR / TEST_MCPT frames with host writes between them (new GPU test)
set -o pipefail
O=gpurun_out/r5/pipehost
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "pipelined" --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -5
