# round 5: trace_stream tuning -- refill threshold (libptx_rf*.so), C1 ReSTIR with dynamic
# batches / the flat walk (measurement build), GI A/B, SIMD utilisation of the streamed walk
set -o pipefail
mkdir -p gpurun_out/r5/stream2
LIBS="libptx.so libptx_rf4.so libptx_rf8.so libptx_rf32.so" REPS=2 TAG=r5/stream2/rf bash tools/ab_libs.sh || exit 1
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L"$'\n'"PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=1"$'\n'"PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=1,FLAT_MIN_INST=1"$'\n'"PTX_LIB_PATH=$L PTX_AB=FLAT_MIN_INST=1" \
  TAG=r5/stream2/c1 BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_env.sh || exit 1
LIBS="libptx.so libptx_alt.so" REPS=1 TAG=r5/stream2/gi BENCH_ARGS="--workload gi --no-configs3" bash tools/ab_libs.sh || exit 1
PTX_AB=TRACE_DYN=1 PTX_LIB_PATH=$L timeout -k 10 300 python3 -u tools/simd_util.py --workload reuse > gpurun_out/r5/stream2/simd_reuse_c3.txt 2>&1 || { echo "simd failed"; tail -5 gpurun_out/r5/stream2/simd_reuse_c3.txt; exit 1; }
grep -A6 "== spatial" gpurun_out/r5/stream2/simd_reuse_c3.txt
