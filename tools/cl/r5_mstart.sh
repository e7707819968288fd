# round 5: the motion start kernel's occupancy (164 B/lane spilled at 3 waves per SIMD)
set -o pipefail
LIBS="libptx.so libptx_m2.so libptx_m4.so libptx_mx.so" REPS=2 TAG=r5/mstart BENCH_ARGS="--no-configs3 --camera-path" bash tools/ab_libs.sh || exit 1
