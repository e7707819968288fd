# round 4 mid-round measurements: the default bench line (CPU baseline + parity window +
# traffic), the moving-camera line, then the configs[3] bands (tools/cl/r4_bands.sh)
set -o pipefail
timeout -k 10 400 python -u bench.py > gpurun_out/r4_mid_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4_mid_bench.log; exit 1; }
tail -n 1 gpurun_out/r4_mid_bench.log
timeout -k 10 300 python -u bench.py --camera-path --no-cpu-baseline --no-configs3 > gpurun_out/r4_mid_motion.log 2>&1 || { echo "motion bench failed"; tail -5 gpurun_out/r4_mid_motion.log; exit 1; }
tail -n 1 gpurun_out/r4_mid_motion.log
bash tools/cl/r4_bands.sh
