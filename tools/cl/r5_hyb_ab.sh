# round 5: the hybrid-shift build against the pre-hybrid kernels (libptx_pre.so, built from the
# commit before) and JOB_STEP_WAVES=4 (libptx_js4.so): headline benches, then per-kernel stats vs pre
set -o pipefail
VARIANTS="pre js4" SKIP_TESTS=1 REPS=2 TAG=r5hyb bash tools/cl/r5_multi_ab.sh || exit 1
TAG=r5hyb_k bash tools/cl/r5_kprof_ab.sh
