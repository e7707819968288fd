# round 5: lane-refill trace walk (trace_stream) -- GPU suite bit-exact, same-box A/B vs the
# batch walk (libptx_alt.so = -DPTX_TRACE_STREAM=0), static + camera-path, SIMD utilisation
set -o pipefail
mkdir -p gpurun_out/r5/stream
timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail 3 --timeout 200 --timeout-method thread > gpurun_out/r5/stream/suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -40 gpurun_out/r5/stream/suite.log; exit 1; }
tail -1 gpurun_out/r5/stream/suite.log
LIBS="libptx.so libptx_alt.so" REPS=2 TAG=r5/stream/ab bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_alt.so" REPS=1 TAG=r5/stream/ab_cam BENCH_ARGS="--no-configs3 --camera-path" bash tools/ab_libs.sh || exit 1
PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so timeout -k 10 300 python3 -u tools/simd_util.py --workload reuse > gpurun_out/r5/stream/simd_reuse_c3.txt 2>&1 || { echo "simd failed"; tail -5 gpurun_out/r5/stream/simd_reuse_c3.txt; exit 1; }
grep -A6 "== spatial" gpurun_out/r5/stream/simd_reuse_c3.txt
