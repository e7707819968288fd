# round 5: early leaf phase thresholds under the streamed walk (headline + C1 ReSTIR)
set -o pipefail
LIBS="libptx.so libptx_k4.so libptx_k16.so libptx_l2.so libptx_l8.so" REPS=2 TAG=r5/leafk BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
LIBS="libptx.so libptx_k4.so libptx_k16.so libptx_l2.so libptx_l8.so" REPS=1 TAG=r5/leafk_c1 BENCH_ARGS="--workload restir --no-configs3" bash tools/ab_libs.sh || exit 1
