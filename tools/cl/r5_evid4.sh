# round 5, final build: GI evidence in its production kernel mode (dynamic batches) + the camera path
set -o pipefail
ROUND=r5 WORKLOADS="gi" bash tools/round_evidence.sh || exit 1
timeout -k 10 300 python3 bench.py --workload gi --camera-path --no-configs3 --no-cpu-baseline > gpurun_out/r5_gicam_final.log 2>&1 || { echo "gi cam failed"; exit 1; }
tail -1 gpurun_out/r5_gicam_final.log | cut -c1-200
