# round 5 (last): logic-kernel occupancy at the static-slot shapes -- start / step kernels at 5 waves
# per SIMD (libptx_lw5.so), GI's spatial start at 4 (libptx_gis4.so), against the measurement build
set -o pipefail
P=$PWD/pathtracerdemo_amd
for wl in restir mcpt gi reuse; do
AB="PTX_LIB_PATH=$P/libptx_ab.so PTX_AB=
PTX_LIB_PATH=$P/libptx_lw5.so PTX_AB="
[ "$wl" = "gi" ] && AB="$AB
PTX_LIB_PATH=$P/libptx_gis4.so PTX_AB="
REPS=2 TAG=r5/occ3/$wl BENCH_ARGS="--workload $wl --no-configs3" AB="$AB" bash tools/ab_env.sh || exit 1
done
echo done
