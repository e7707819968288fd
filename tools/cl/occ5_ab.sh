# trace at 5 waves per SIMD (the flattened walk spills 40 B/lane there) vs 4, per workload
set -o pipefail
AB=$'PTX_AB=\nPTX_AB=TRACE_OCC=5'
AB="$AB" REPS=2 TAG=occ5_reuse BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
AB="$AB" REPS=1 TAG=occ5_gi BENCH_ARGS="--no-configs3 --workload gi" bash tools/ab_env.sh || exit 1
AB="$AB" REPS=1 TAG=occ5_restir BENCH_ARGS="--no-configs3 --workload restir" bash tools/ab_env.sh || exit 1
AB="$AB" REPS=1 TAG=occ5_mcpt BENCH_ARGS="--no-configs3 --workload mcpt" bash tools/ab_env.sh || exit 1
AB="$AB" REPS=1 TAG=occ5_furn_gi BENCH_ARGS="--no-configs3 --workload gi --scene c3_furnished" bash tools/ab_env.sh || exit 1
