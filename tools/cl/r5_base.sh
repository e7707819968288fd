# round 5: baseline profiles before the trace / motion work -- kernel stats of the static headline
# and of the moving-camera bench, the camera-path bench line, SIMD utilisation (measurement build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5/base
mkdir -p $O/static $O/motion
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/static -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-configs3 --steps 10 --warmup 3 > $O/static/bench.log 2>&1 || { echo "static prof failed"; tail -5 $O/static/bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/motion -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-configs3 --camera-path --steps 10 --warmup 3 > $O/motion/bench.log 2>&1 || { echo "motion prof failed"; tail -5 $O/motion/bench.log; exit 1; }
cd $R
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-configs3 --camera-path > $O/camera_path.log 2>&1 || { echo "camera bench failed"; tail -5 $O/camera_path.log; exit 1; }
tail -1 $O/camera_path.log | cut -c1-300
PTX_LIB_PATH=$R/pathtracerdemo_amd/libptx_ab.so timeout -k 10 300 python3 -u tools/simd_util.py --workload reuse > $O/simd_reuse_c3.txt 2>&1 || { echo "simd failed"; tail -5 $O/simd_reuse_c3.txt; exit 1; }
grep -A6 "== spatial" $O/simd_reuse_c3.txt
