# round 5: early leaf phase K / L under the streamed walk, second sweep (headline)
set -o pipefail
LIBS="libptx.so libptx_k16.so libptx_k24.so libptx_k32.so libptx_k16l2.so libptx_k16l6.so" REPS=2 TAG=r5/leafk2 BENCH_ARGS="--no-configs3" bash tools/ab_libs.sh || exit 1
