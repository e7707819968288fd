# the flattened walk at 6 waves per SIMD (80 VGPRs, 136 B/lane spilled) vs 5 (PTX_AB=TRACE_OCC=6)
set -o pipefail
PTX_AB=TRACE_OCC=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/occ6_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/occ6_tests.log; exit 1; }
tail -1 gpurun_out/occ6_tests.log
AB=$'PTX_AB=\nPTX_AB=TRACE_OCC=6'
AB="$AB" REPS=2 TAG=ab_occ6 BENCH_ARGS="" bash tools/ab_env.sh || exit 1
for f in gpurun_out/ab_occ6/run_*.log; do grep '^{' $f | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["env"], "configs3", d["configs3_one_gpu"]["value"])'; done
AB="$AB" REPS=1 TAG=ab_occ6_f BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
AB="$AB" REPS=1 TAG=ab_occ6_gi BENCH_ARGS="--no-configs3 --workload gi" bash tools/ab_env.sh || exit 1
