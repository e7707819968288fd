# round 5: static vs dynamic trace slots for 2- and 4-way bands of configs[3] (each alone, proxy)
set -o pipefail
mkdir -p gpurun_out/r5/bands4
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
for W in 2 4; do
for T in "" ",TRACE_DYN=1"; do
PTX_AB=HALO_PROXY_US=110$T timeout -k 10 400 python -u tools/band_alone.py --world $W > gpurun_out/r5/bands4/w$W$T.jsonl 2> gpurun_out/r5/bands4/err.txt || { echo "w$W failed"; tail -5 gpurun_out/r5/bands4/err.txt; exit 1; }
echo "world $W $T: $(cut -c1-300 gpurun_out/r5/bands4/w$W$T.jsonl)"
done; done
