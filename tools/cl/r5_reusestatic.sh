# round 5: GI on static slots + 2 sequences (GI / band / loopback tests, GI bench with parity, moving
# GI); then the headline's trace slots and segments at the pipelined frames (measurement build)
set -o pipefail
O=gpurun_out/r5/reusestatic
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_gi.py tests/test_gpu_bands.py tests/test_gpu_loopback.py -m gpu -q --maxfail 3 --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "GI tests failed"; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 bench.py --workload gi --no-configs3 > $O/gi.log 2>&1 || { echo "bench failed"; tail -20 $O/gi.log; exit 1; }
tail -1 $O/gi.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("gi", d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("parity"))'
timeout -k 10 400 python3 bench.py --workload gi --no-configs3 --camera-path --no-cpu-baseline > $O/gicam.log 2>&1 || { echo "cam bench failed"; tail -20 $O/gicam.log; exit 1; }
tail -1 $O/gicam.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("gi cam", d["value"], d["ms_per_step"], d["roofline"]["frac"])'
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=0
PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=0,SEG_PX=1792
PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=0,SEG_PX=1792,PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1792" REPS=2 TAG=r5/reusestatic/ab BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
echo done
