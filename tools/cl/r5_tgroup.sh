# round 5: trace workgroups over groups of consecutive segments (static slots, streamed walk):
# parity subset, then C1 ReSTIR / MCPT and a band with TRACE_GROUP = 1..4 (measurement build)
set -o pipefail
L=$PWD/pathtracerdemo_amd/libptx_ab.so
PTX_LIB_PATH=$L PTX_AB=TRACE_GROUP=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gi.py tests/test_gpu_bands.py -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/r5_tgroup_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5_tgroup_tests.log; exit 1; }
tail -1 gpurun_out/r5_tgroup_tests.log
AB=""
for k in "" "TRACE_GROUP=2" "TRACE_GROUP=3" "TRACE_GROUP=4"; do AB+="PTX_LIB_PATH=$L PTX_AB=$k"$'\n'; done
AB="$AB" TAG=r5/tgroup_c1 BENCH_ARGS="--no-configs3 --workload restir" bash tools/ab_env.sh || exit 1
AB="$AB" TAG=r5/tgroup_mcpt BENCH_ARGS="--no-configs3 --workload mcpt" bash tools/ab_env.sh || exit 1
export PTX_LIB_PATH=$L
P=HALO_PROXY_US=110
timeout -k 10 600 python -u tools/band_knobs.py --band 895,1059 --ab "$P" "$P,TRACE_GROUP=2" "$P,TRACE_GROUP=3" "$P,TRACE_GROUP=4" "$P" || exit 1
