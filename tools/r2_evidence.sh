#!/usr/bin/env bash
# Round-2 evidence in one GPU call: round_evidence.sh for every workload (rocprofv3 trace +
# stats, PMC FETCH_SIZE / WRITE_SIZE, bench line with CPU baselines), then configs[3] at 4K on
# one GPU and the furnished scene.  Then, here: ROUND=r2 bash tools/collect_profiles.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
ROUND=${ROUND:-r2}
ROUND=$ROUND WORKLOADS="${WORKLOADS:-reuse restir mcpt gi}" bash tools/round_evidence.sh || exit 1
mkdir -p gpurun_out/strong_4k_$ROUND
timeout -k 10 300 python3 bench.py --frame 3840x2160 --steps 8 --warmup 2 > gpurun_out/strong_4k_$ROUND/bench_1gpu.log 2>&1 \
    || { echo "4k 1gpu failed"; exit 1; }
echo "4k: $(tail -n 1 gpurun_out/strong_4k_$ROUND/bench_1gpu.log | cut -c1-160)"
timeout -k 10 300 python3 bench.py --scene c3_furnished --steps 15 --warmup 3 > gpurun_out/strong_4k_$ROUND/bench_furnished.log 2>&1 \
    || { echo "furnished failed"; exit 1; }
echo "furnished: $(tail -n 1 gpurun_out/strong_4k_$ROUND/bench_furnished.log | cut -c1-160)"
