# node-pair fetch through a buffer resource (PTX_NODE_BUF), wjob_step gathers issued beside the job
# header (PTX_JOB_PREFETCH), surface_at's M^-1 read once (PTX_SURF_HOIST), branch-free wspatial_start
# gathers (PTX_START_FLAT_LOADS): GPU suite on the new
# build, then same-box A/B of new / HEAD / one-switch-off builds on the headline, new vs HEAD furnished
set -o pipefail
P=$PWD/pathtracerdemo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/nb_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/nb_tests.log; exit 1; }
tail -1 gpurun_out/nb_tests.log
L=""; for v in libptx.so libptx_head.so libptx_nb0.so libptx_pf0.so libptx_sh0.so libptx_sl0.so; do L+="PTX_LIB_PATH=$P/$v"$'\n'; done
AB="$L" REPS=2 TAG=ab_nb BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$P/libptx.so"$'\n'"PTX_LIB_PATH=$P/libptx_head.so" REPS=1 TAG=ab_nb_f BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
