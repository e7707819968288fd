# round 5 (last): trace occupancy for a configs[3] band (rows 895-1061, alone, 110 us proxy)
set -o pipefail
mkdir -p gpurun_out/r5/bandocc
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
P=HALO_PROXY_US=110
timeout -k 10 600 python -u tools/band_knobs.py --band 895,1061 --ab "$P" "$P,TRACE_OCC=4" "$P,TRACE_OCC=6" "$P,TRACE_DYN=1" "$P" > gpurun_out/r5/bandocc/mid.jsonl 2> gpurun_out/r5/bandocc/mid.err || { echo "sweep failed"; tail -5 gpurun_out/r5/bandocc/mid.err; exit 1; }
cat gpurun_out/r5/bandocc/mid.jsonl
