# the spatial pass's shift jobs in slot planes (job id = pix + slot * npix: a wave's jobs fill whole
# 128-byte lines of the SoA state) against pixel-major ids (PTX_AB=JOB_PLANES=0): GPU suite, then
# same-box A/B on the headline (3 reps) and the furnished scene
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/jplane_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/jplane_tests.log; exit 1; }
tail -1 gpurun_out/jplane_tests.log
AB=$'PTX_AB=\nPTX_AB=JOB_PLANES=0' REPS=3 TAG=ab_jplane BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=JOB_PLANES=0' REPS=1 TAG=ab_jplane_f BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
