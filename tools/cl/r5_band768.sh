# round 5 (late): a configs[3] band (rows 895-1061, alone, 110 us proxy) at 768-pixel segments
set -o pipefail
mkdir -p gpurun_out/r5/band768
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
P=HALO_PROXY_US=110
timeout -k 10 600 python -u tools/band_knobs.py --band 895,1061 --ab "$P" "$P,SEG_PX=768" "$P" "$P,SEG_PX=768" > gpurun_out/r5/band768/mid.jsonl 2> gpurun_out/r5/band768/mid.err || { echo "sweep failed"; tail -5 gpurun_out/r5/band768/mid.err; exit 1; }
cat gpurun_out/r5/band768/mid.jsonl
