# GPU suite + default bench line + 8-band re-cut timing (one band per process)
set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ca_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ca_tests.log; exit 1; }
tail -1 gpurun_out/ca_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/ca_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ca_bench.log; exit 1; }
grep '^{' gpurun_out/ca_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["configs3_one_gpu"]["value"], d["cpu_baseline"]["value"])'
if [ "${RECUT:-1}" = "1" ]; then
timeout -k 10 600 python -u tools/band_alone.py --world 8 --recut 3 > gpurun_out/ca_recut.log 2>&1 || { echo "recut failed"; exit 1; }
tail -1 gpurun_out/ca_recut.log | cut -c1-400
fi
