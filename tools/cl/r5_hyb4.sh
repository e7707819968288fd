# round 5: hybrid shift v2 (full GetSurface of the stored vertex in job_emit) vs v2pos (default:
# position + roughness only there), each at 5 / 4 job-step waves, against the pre-hybrid kernels
set -o pipefail
P=$PWD/pathtracerdemo_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_bands.py -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/r5hyb4_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/r5hyb4_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r5hyb4_tests.log)"
VARIANTS="pre pj4 v2 v2j4" SKIP_TESTS=1 REPS=2 TAG=r5hyb4 bash tools/cl/r5_multi_ab.sh
