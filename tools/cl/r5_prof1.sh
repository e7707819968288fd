# round 5: evidence at the streamed trace walk -- kernel stats of the static headline (the
# roofline's trace_queue) and of the moving camera, SIMD utilisation by region (measurement build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5/prof1
mkdir -p $O/reuse $O/motion
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/reuse -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-configs3 --steps 10 --warmup 3 > $O/reuse/bench.log 2>&1 || { echo "static prof failed"; tail -5 $O/reuse/bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/motion -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-configs3 --camera-path --steps 10 --warmup 3 > $O/motion/bench.log 2>&1 || { echo "motion prof failed"; tail -5 $O/motion/bench.log; exit 1; }
cd $R
PTX_LIB_PATH=$R/pathtracerdemo_amd/libptx_ab.so timeout -k 10 300 python3 -u tools/simd_util.py --workload reuse > $O/simd_reuse_c3.txt 2>&1 || { echo "simd failed"; tail -5 $O/simd_reuse_c3.txt; exit 1; }
PTX_LIB_PATH=$R/pathtracerdemo_amd/libptx_ab.so timeout -k 10 300 python3 -u tools/simd_util.py --workload restir > $O/simd_restir_c1.txt 2>&1 || { echo "simd failed"; exit 1; }
grep -A6 "== spatial" $O/simd_reuse_c3.txt
grep -A6 "== init" $O/simd_restir_c1.txt | head -7
