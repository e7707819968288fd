# round 4: GPU suite, A/B of the LDS transmission lookup (alt = PTX_LDS_TRANS=0), the bench
# line (CPU baseline + parity window + traffic), the moving-camera line, then the headline's
# round-4 rocprof / PMC evidence (reuse)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_mid3_tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -40 gpurun_out/r4_mid3_tests.log; exit 1; }
tail -1 gpurun_out/r4_mid3_tests.log
REPS=2 TAG=r4_ldstrans bash tools/cl/ab_alt.sh || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r4_mid_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4_mid_bench.log; exit 1; }
tail -n 1 gpurun_out/r4_mid_bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --camera-path --no-cpu-baseline --no-configs3 > gpurun_out/r4_mid_motion.log 2>&1 || { echo "motion bench failed"; tail -5 gpurun_out/r4_mid_motion.log; exit 1; }
tail -n 1 gpurun_out/r4_mid_motion.log | cut -c1-400
WLS=reuse bash tools/cl/evidence_r4.sh
