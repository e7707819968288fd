# round 5, final build: evidence for reuse + gi (rocprof stats, PMC, bench lines), the moving-camera
# bench line, SIMD utilisation at this build
set -o pipefail
ROUND=r5 WORKLOADS="reuse gi" bash tools/round_evidence.sh || exit 1
mkdir -p gpurun_out/r5/final
timeout -k 10 300 python3 bench.py --no-configs3 --no-cpu-baseline --camera-path > gpurun_out/r5/final/camera_path.log 2>&1 || { echo "camera failed"; exit 1; }
tail -1 gpurun_out/r5/final/camera_path.log | cut -c1-200
PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so timeout -k 10 300 python3 -u tools/simd_util.py --workload reuse > gpurun_out/r5/final/simd_reuse_c3.txt 2>&1 || { echo "simd failed"; exit 1; }
grep -A6 "== spatial" gpurun_out/r5/final/simd_reuse_c3.txt
