# round 5: ReSTIR defaults (pipelined, ~1150 segments, 2 sequences per context): ReSTIR GPU tests
# incl. the 1080p pipelined window, then the default restir bench line (with its parity window)
set -o pipefail
O=gpurun_out/r5/piperestir6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_present.py tests/test_gpu_cull.py tests/test_gpu_large_tables.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 400 python3 bench.py --workload restir --no-configs3 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("parity"))'
echo done
