# round 5: hybrid-shift job layouts: v3 (default: the hybrid work moved into job_emit, steps only
# check the connection) and v4 (one vertex per loop iteration in job_emit), each at 5 / 4 job-step
# waves, against the pre-hybrid kernels; reuse GPU tests on v3 and v4 first
set -o pipefail
P=$PWD/pathtracerdemo_amd
for v in cur v4; do
  lib=""; [ "$v" != cur ] && lib=$P/libptx_$v.so
  PTX_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_bands.py -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/r5hyb3_tests_$v.log 2>&1 \
    || { echo "tests $v failed"; tail -30 gpurun_out/r5hyb3_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r5hyb3_tests_$v.log)"
done
VARIANTS="pre v3j4 v4 v4j4" SKIP_TESTS=1 REPS=2 TAG=r5hyb3 bash tools/cl/r5_multi_ab.sh
