# pipelined band frames: GPU suite, then per-band times alone (tools/band_alone.py) with and
# without band pipelining, and with the halo overlap
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bp_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/bp_tests.log; exit 1; }
tail -1 gpurun_out/bp_tests.log
timeout -k 10 200 python -u tools/band_alone.py --world 8 > gpurun_out/bp_alone_pipe.log 2>&1 || { echo "alone pipe failed"; tail -20 gpurun_out/bp_alone_pipe.log; exit 1; }
echo "pipe: $(tail -1 gpurun_out/bp_alone_pipe.log)"
PTX_AB=PIPELINE_BANDS=0 timeout -k 10 200 python -u tools/band_alone.py --world 8 > gpurun_out/bp_alone_nopipe.log 2>&1 || { echo "alone nopipe failed"; exit 1; }
echo "nopipe: $(tail -1 gpurun_out/bp_alone_nopipe.log)"
timeout -k 10 200 python -u tools/band_alone.py --world 8 --overlap > gpurun_out/bp_alone_pipe_ov.log 2>&1 || { echo "alone overlap failed"; exit 1; }
echo "pipe+overlap: $(tail -1 gpurun_out/bp_alone_pipe_ov.log)"
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/bp_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bp_bench.log; exit 1; }
grep '^{' gpurun_out/bp_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d.get("configs3_one_gpu"))'
