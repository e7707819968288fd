# round 5 (late): GI back on one front sequence per context -- GI / band / loopback tests, GI evidence
set -o pipefail
O=gpurun_out/r5/evid6
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_gi.py tests/test_gpu_bands.py tests/test_gpu_loopback.py -m gpu -q --maxfail 3 --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "GI tests failed"; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ROUND=r5 WORKLOADS="gi" bash tools/round_evidence.sh || exit 1
timeout -k 10 400 python3 bench.py --workload gi --no-configs3 --camera-path --no-cpu-baseline > $O/gicam.log 2>&1 || { echo "cam bench failed"; tail -20 $O/gicam.log; exit 1; }
tail -1 $O/gicam.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("gi cam", d["value"], d["ms_per_step"], d["roofline"]["frac"])'
