# round 5 (last): the configs[3] bands at the last build, each alone with the 110 us exchange proxy --
# the previous re-cut, then one more measured re-cut; and the one-GPU 4K frame of the same build
set -o pipefail
O=gpurun_out/r5/bands5
mkdir -p $O
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
B='[[0, 572], [572, 750], [750, 895], [895, 1059], [1059, 1281], [1281, 1534], [1534, 1778], [1778, 2160]]'
PTX_AB=HALO_PROXY_US=110 timeout -k 10 600 python -u tools/band_alone.py --world 8 --bands "$B" --recut 1 > $O/recut.jsonl 2> $O/err.txt || { echo "bands failed"; tail -5 $O/err.txt; exit 1; }
cut -c1-400 $O/recut.jsonl
