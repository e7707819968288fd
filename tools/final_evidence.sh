#!/usr/bin/env bash
# Round-end evidence in one GPU call: round_evidence.sh for every workload, then configs[3]'s
# strong-scaling lines (one 3840x2160 frame on one GPU; the same frame as 2 gloo ranks
# sharing it -- a rehearsal of the band + halo path).  usage: ROUND=r1 bash tools/final_evidence.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
ROUND=${ROUND:-r1}
WORKLOADS="${WORKLOADS:-reuse restir mcpt gi}" bash tools/round_evidence.sh || exit 1
mkdir -p gpurun_out/strong_4k
timeout -k 10 300 python3 bench.py --frame 3840x2160 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/strong_4k/bench_1gpu.log 2>&1 || { echo "4k 1gpu failed"; exit 1; }
echo "4k: $(tail -n 1 gpurun_out/strong_4k/bench_1gpu.log | cut -c1-160)"
PTX_DIST_BACKEND=gloo PTX_FORCE_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --frame 3840x2160 --steps 5 \
    --warmup 2 --no-cpu-baseline > gpurun_out/strong_4k/bench_2ranks.log 2>&1 || { echo "4k 2 ranks failed"; exit 1; }
echo "4k x2: $(grep '^{' gpurun_out/strong_4k/bench_2ranks.log | tail -n 1 | cut -c1-160)"
