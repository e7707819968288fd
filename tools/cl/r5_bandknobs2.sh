# round 5: band switches at static trace slots (measurement build, proxy): trace occupancy, segment size
set -o pipefail
mkdir -p gpurun_out/r5/bandknobs2
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
P=HALO_PROXY_US=110
for b in 895,1059 0,572; do
timeout -k 10 600 python -u tools/band_knobs.py --band $b --ab "$P" "$P,TRACE_OCC=4" "$P,SEG_PX=256" "$P,TRACE_OCC=4,SEG_PX=256" "$P,PIPE_BACK_STREAMS=1" "$P" > gpurun_out/r5/bandknobs2/b$b.jsonl 2> gpurun_out/r5/bandknobs2/err.txt || { echo "sweep failed"; tail -5 gpurun_out/r5/bandknobs2/err.txt; exit 1; }
cat gpurun_out/r5/bandknobs2/b$b.jsonl
done
