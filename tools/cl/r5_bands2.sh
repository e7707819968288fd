# round 5: the re-cut configs[3] bands alone with the proxy: dynamic vs static trace batches
# (measurement build), and the headline with static batches
set -o pipefail
mkdir -p gpurun_out/r5/bands2
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
B='[[0, 570], [570, 749], [749, 895], [895, 1061], [1061, 1282], [1282, 1528], [1528, 1765], [1765, 2160]]'
PTX_AB=HALO_PROXY_US=110 timeout -k 10 400 python -u tools/band_alone.py --world 8 --bands "$B" > gpurun_out/r5/bands2/dyn.jsonl 2> gpurun_out/r5/bands2/err.txt || { echo "dyn failed"; tail -5 gpurun_out/r5/bands2/err.txt; exit 1; }
cut -c1-300 gpurun_out/r5/bands2/dyn.jsonl
PTX_AB=HALO_PROXY_US=110,TRACE_DYN=0 timeout -k 10 400 python -u tools/band_alone.py --world 8 --bands "$B" > gpurun_out/r5/bands2/static.jsonl 2>> gpurun_out/r5/bands2/err.txt || { echo "static failed"; exit 1; }
cut -c1-300 gpurun_out/r5/bands2/static.jsonl
AB="PTX_LIB_PATH=$PTX_LIB_PATH PTX_AB="$'\n'"PTX_LIB_PATH=$PTX_LIB_PATH PTX_AB=TRACE_DYN=0" REPS=2 TAG=r5/bands2/hd BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
