# round 5: C1 ReSTIR / MCPT segment size under the streamed walk on static slots (measurement build)
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB=""
for k in "" "SEG_PX=1024" "SEG_PX=1536" "SEG_PX=2048" "SEG_PX=3072"; do AB+="PTX_LIB_PATH=$L PTX_AB=$k"$'\n'; done
AB="$AB" TAG=r5/c1seg BENCH_ARGS="--no-configs3 --workload restir" bash tools/ab_env.sh || exit 1
AB="$AB" TAG=r5/c1seg_m BENCH_ARGS="--no-configs3 --workload mcpt" bash tools/ab_env.sh || exit 1
