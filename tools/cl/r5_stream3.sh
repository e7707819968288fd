# round 5: trace_stream on static slots too (GI, ReSTIR, MCPT) -- GPU suite, refill threshold
# 24 / 32 / 48, GI / C1 ReSTIR / MCPT vs the batch walk, C1 with the flat walk (measurement build)
set -o pipefail
mkdir -p gpurun_out/r5/stream3
timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail 3 --timeout 200 --timeout-method thread > gpurun_out/r5/stream3/suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -40 gpurun_out/r5/stream3/suite.log; exit 1; }
tail -1 gpurun_out/r5/stream3/suite.log
LIBS="libptx.so libptx_rf24.so libptx_rf48.so libptx_alt.so" REPS=2 TAG=r5/stream3/rf bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_alt.so" REPS=1 TAG=r5/stream3/gi BENCH_ARGS="--workload gi --no-configs3" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_alt.so" REPS=1 TAG=r5/stream3/mcpt BENCH_ARGS="--workload mcpt --no-configs3" bash tools/ab_libs.sh || exit 1
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L"$'\n'"PTX_LIB_PATH=$L PTX_AB=FLAT_MIN_INST=1"$'\n'"PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_alt.so" \
  TAG=r5/stream3/c1 BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB=FLAT_MIN_INST=1" TAG=r5/stream3/c1m BENCH_ARGS="--workload mcpt --no-configs3" bash tools/ab_env.sh || exit 1
