# identity instances' ray transform as x + 0 in the flattened walk (PTX_TRACE_IDENT): GPU suite,
# then same-box A/B against -DPTX_TRACE_IDENT=0 (headline + its configs3_one_gpu 4K line, furnished)
set -o pipefail
P=$PWD/pathtracerdemo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ident_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ident_tests.log; exit 1; }
tail -1 gpurun_out/ident_tests.log
AB="PTX_LIB_PATH=$P/libptx.so"$'\n'"PTX_LIB_PATH=$P/libptx_id0.so" REPS=2 TAG=ab_ident bash tools/ab_env.sh || exit 1
for f in gpurun_out/ab_ident/run_*.log; do grep '^{' $f | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("4K one GPU", d["configs3_one_gpu"]["value"])'; done
AB="PTX_LIB_PATH=$P/libptx.so"$'\n'"PTX_LIB_PATH=$P/libptx_id0.so" REPS=1 TAG=ab_ident_f BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
