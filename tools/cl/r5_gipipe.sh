# round 5: ReSTIR GI frames pipelined (two in flight, as the DI reuse pipeline) -- GI / band /
# loopback GPU tests bit-exact, then GI bench vs unpipelined (measurement build), still + moving
set -o pipefail
mkdir -p gpurun_out/r5/gipipe
timeout -k 10 500 python -u -m pytest tests/test_gpu_gi.py tests/test_gpu_bands.py tests/test_gpu_loopback.py -m gpu -q --maxfail 3 --timeout 240 --timeout-method thread > gpurun_out/r5/gipipe/tests.log 2>&1 \
    || { echo "GI tests failed"; tail -60 gpurun_out/r5/gipipe/tests.log; exit 1; }
tail -1 gpurun_out/r5/gipipe/tests.log
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=PIPELINE_FRAMES=0" REPS=2 TAG=r5/gipipe/ab BENCH_ARGS="--workload gi --no-configs3" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=PIPELINE_FRAMES=0" TAG=r5/gipipe/cam BENCH_ARGS="--workload gi --no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
