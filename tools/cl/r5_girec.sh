# round 5: GI spatial pass reading per-pixel surface records (wgi_records) instead of computing
# GetSurface per shift job -- GI / band / loopback GPU tests bit-exact, then A/B GI_RECORDS on / off
# (measurement build), still + moving camera, and the kernel stats of the GI bench
set -o pipefail
mkdir -p gpurun_out/r5/girec
timeout -k 10 500 python -u -m pytest tests/test_gpu_gi.py tests/test_gpu_bands.py tests/test_gpu_loopback.py -m gpu -q --maxfail 3 --timeout 240 --timeout-method thread > gpurun_out/r5/girec/tests.log 2>&1 \
    || { echo "GI tests failed"; tail -60 gpurun_out/r5/girec/tests.log; exit 1; }
tail -1 gpurun_out/r5/girec/tests.log
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=GI_RECORDS=0" REPS=3 TAG=r5/girec/ab BENCH_ARGS="--workload gi --no-configs3" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB="$'\n'"PTX_LIB_PATH=$L PTX_AB=GI_RECORDS=0" TAG=r5/girec/cam BENCH_ARGS="--workload gi --no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/girec/prof -o gi -- python3 bench.py --workload gi --no-configs3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5/girec/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/r5/girec/prof.log; exit 1; }
echo done
