# round 5: band handles on static trace slots -- GPU suite, one measured re-cut of the bands with
# the proxy (measurement build), the default bench line (smoke included)
set -o pipefail
bash tools/cl/r5_suite.sh || exit 1
mkdir -p gpurun_out/r5/bands3
B='[[0, 570], [570, 749], [749, 895], [895, 1061], [1061, 1282], [1282, 1528], [1528, 1765], [1765, 2160]]'
PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so PTX_AB=HALO_PROXY_US=110 timeout -k 10 600 python -u tools/band_alone.py --world 8 --bands "$B" --recut 1 > gpurun_out/r5/bands3/recut.jsonl 2> gpurun_out/r5/bands3/err.txt || { echo "recut failed"; tail -5 gpurun_out/r5/bands3/err.txt; exit 1; }
cut -c1-300 gpurun_out/r5/bands3/recut.jsonl
