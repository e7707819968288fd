# round 5: ReSTIR (no reuse) frames pipelined -- GPU suite, then A/B PIPE_RESTIR on / off on the
# C1 ReSTIR workload (measurement build)
set -o pipefail
mkdir -p gpurun_out/r5/piperestir
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/piperestir/suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -60 gpurun_out/r5/piperestir/suite.log; exit 1; }
tail -1 gpurun_out/r5/piperestir/suite.log
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=PIPE_RESTIR=0" REPS=3 TAG=r5/piperestir/ab BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_env.sh || exit 1
echo done
