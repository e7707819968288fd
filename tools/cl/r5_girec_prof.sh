# round 5: kernel stats of the GI bench with and without the spatial pass's surface records
set -o pipefail
mkdir -p gpurun_out/r5/girec
L=$PWD/pathtracerdemo_amd/libptx_ab.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 1 0; do
  PTX_LIB_PATH=$L PTX_AB=GI_RECORDS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/girec/prof$v -o run --output-format csv -- python3 bench.py --workload gi --no-configs3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5/girec/prof$v.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/r5/girec/prof$v.log; exit 1; }
done
echo done
