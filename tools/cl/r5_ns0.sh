# round 5 (late): timing diagnostic -- the moving-camera frame with the motion start kernel's slot 0
# (the canonical sample at home) skipped (libptx_ns0.so, wrong results) against the default: how much
# of wtmotion_start is the rarely active slot-0 iteration
set -o pipefail
O=gpurun_out/r5/ns0
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ab ns0; do
  PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-configs3 --camera-path --steps 10 --warmup 3 > $O/$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/$v.log; exit 1; }
  grep -E "wtmotion_start|wtmotion_combine" $O/$v/run_kernel_stats.csv | cut -d, -f1-4
done
