# the flattened walk at 5 waves per SIMD by default: GPU suite, then same-box A/B against 4
# (PTX_AB=TRACE_OCC=4) on the headline (configs[3]'s 4K frame included), GI and the furnished C3
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/occ5_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/occ5_tests.log; exit 1; }
tail -1 gpurun_out/occ5_tests.log
AB=$'PTX_AB=\nPTX_AB=TRACE_OCC=4'
AB="$AB" REPS=2 TAG=occ5c_reuse BENCH_ARGS="" bash tools/ab_env.sh || exit 1
for f in gpurun_out/occ5c_reuse/run_*.log; do grep '^{' $f | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["env"], "configs3", d["configs3_one_gpu"]["value"])'; done
AB="$AB" REPS=1 TAG=occ5c_furn BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
