# round 4: GPU suite, A/B of the LDS transmission lookup (alt = PTX_LDS_TRANS=0), then the
# mid-round measurements (tools/cl/r4_mid.sh: bench line, moving camera, configs[3] bands)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_mid2_tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -40 gpurun_out/r4_mid2_tests.log; exit 1; }
tail -1 gpurun_out/r4_mid2_tests.log
REPS=2 TAG=r4_ldstrans bash tools/cl/ab_alt.sh || exit 1
bash tools/cl/r4_mid.sh
