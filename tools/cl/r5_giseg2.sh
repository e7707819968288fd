# round 5: GI at ~1150 segments (1792 px at 1080p): GI / band / loopback GPU tests, default GI bench
# line (parity window) and the moving GI camera
set -o pipefail
O=gpurun_out/r5/giseg2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_gi.py tests/test_gpu_bands.py tests/test_gpu_loopback.py -m gpu -q --maxfail 3 --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "GI tests failed"; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 bench.py --workload gi --no-configs3 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("parity"))'
timeout -k 10 400 python3 bench.py --workload gi --no-configs3 --camera-path --no-cpu-baseline > $O/cam.log 2>&1 || { echo "cam bench failed"; tail -20 $O/cam.log; exit 1; }
tail -1 $O/cam.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])'
echo done
