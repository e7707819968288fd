# round 4: SIMD utilisation per traversal region (the headline's spatial pass etc.) at the
# round's kernels, and the restir workload for C1
set -o pipefail
mkdir -p gpurun_out/r4_simd
timeout -k 10 300 python -u tools/simd_util.py --workload reuse > gpurun_out/r4_simd/reuse_c3.txt 2>&1 || { echo "simd reuse failed"; tail -5 gpurun_out/r4_simd/reuse_c3.txt; exit 1; }
grep -A6 "== spatial" gpurun_out/r4_simd/reuse_c3.txt
timeout -k 10 300 python -u tools/simd_util.py --workload restir > gpurun_out/r4_simd/restir_c1.txt 2>&1 || { echo "simd restir failed"; exit 1; }
grep -A6 "== init" gpurun_out/r4_simd/restir_c1.txt | head -8
