# fresh shift jobs keep rSeed[1] in their state (no reservoir gather in wjob_step's fresh-job
# load) + the temporal combine with four lanes per pixel (PTX_AB=TCOMBINE_QUAD=0: one lane):
# GPU reuse / bands suites, then same-box A/B against the previous build (libptx_base.so)
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_bands.py tests/test_gpu_debug_fill.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tquad_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tquad_tests.log; exit 1; }
tail -1 gpurun_out/tquad_tests.log
P=$PWD/pathtracerdemo_amd
AB="PTX_LIB_PATH=$P/libptx.so"$'\n'"PTX_LIB_PATH=$P/libptx.so PTX_AB=TCOMBINE_QUAD=0"$'\n'"PTX_LIB_PATH=$P/libptx_base.so"
AB="$AB" REPS=3 TAG=ab_tquad BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
AB="$AB" REPS=1 TAG=ab_tquad_f BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
