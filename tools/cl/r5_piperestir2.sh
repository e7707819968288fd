# round 5: pipelined ReSTIR frames with static trace slots (default) against dynamic batches
# (TRACE_DYN=1) and one frame at a time (PIPE_RESTIR=0); ReSTIR GPU tests first
set -o pipefail
mkdir -p gpurun_out/r5/piperestir2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_present.py tests/test_gpu_cull.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/piperestir2/tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -60 gpurun_out/r5/piperestir2/tests.log; exit 1; }
tail -1 gpurun_out/r5/piperestir2/tests.log
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=PIPE_RESTIR=0"$'\n'"PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=1" REPS=3 TAG=r5/piperestir2/ab BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_env.sh || exit 1
echo done
