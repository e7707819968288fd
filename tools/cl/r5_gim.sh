# round 5: GI motion tests (whole image, bands, loopback communicator)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 500 python -u -m pytest tests/test_gpu_gi.py tests/test_gpu_bands.py tests/test_gpu_loopback.py -m gpu -v --maxfail 4 --timeout 240 --timeout-method thread > gpurun_out/r5/gim.log 2>&1 \
    || { echo "GI motion tests failed"; tail -80 gpurun_out/r5/gim.log; exit 1; }
tail -3 gpurun_out/r5/gim.log
