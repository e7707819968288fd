# round 5: pipelined TEST_MCPT defaults (static slots, 1792 px, 2 sequences per context): the whole
# GPU suite, the default MCPT bench line (parity window); GI launch-shape switches at 1792 px
set -o pipefail
O=gpurun_out/r5/pipemcpt3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -60 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 400 python3 bench.py --workload mcpt --no-configs3 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("parity"))'
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=0
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=2,TRACE_DYN=0" REPS=2 TAG=r5/pipemcpt3/gi BENCH_ARGS="--workload gi --no-configs3" bash tools/ab_env.sh || exit 1
echo done
