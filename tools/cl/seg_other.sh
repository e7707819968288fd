# segment size of the other pipelines at 1080p (default 768 px)
set -o pipefail
for wl in gi restir mcpt; do
  AB=$'PTX_AB=\nPTX_AB=SEG_PX=512\nPTX_AB=SEG_PX=1024' REPS=1 TAG=segother_$wl BENCH_ARGS="--no-configs3 --workload $wl" bash tools/ab_env.sh || exit 1
done
