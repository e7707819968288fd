# reuse segments scaled with the band (512 .. 4096 px): GPU suite, default bench (1080p + the 4K
# one-GPU frame), configs[3]'s 8 bands re-cut 3 times, each alone
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/segscale_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/segscale_tests.log; exit 1; }
tail -1 gpurun_out/segscale_tests.log
for rep in 1 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/segscale_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/segscale_bench.log; exit 1; }
grep '^{' gpurun_out/segscale_bench.log | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["configs3_one_gpu"]["value"])'
done
timeout -k 10 600 python -u tools/band_alone.py --world 8 --recut 3 > gpurun_out/segscale_recut.log 2>&1 || { echo "recut failed"; tail -5 gpurun_out/segscale_recut.log; exit 1; }
tail -n 1 gpurun_out/segscale_recut.log | cut -c1-300
