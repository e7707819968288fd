# round 5 (late): a configs[3] band (rows 895-1061, alone, 110 us exchange proxy) with the front
# passes in 2 launch sequences per context (the whole-image default since the static-slot change) vs 1
set -o pipefail
mkdir -p gpurun_out/r5/bandps
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
P=HALO_PROXY_US=110
timeout -k 10 900 python -u tools/band_knobs.py --band 895,1061 --ab "$P" "$P,PIPE_STREAMS=1" "$P,PIPE_STREAMS=2,SEG_PX=768" "$P" "$P,PIPE_STREAMS=1" > gpurun_out/r5/bandps/mid.jsonl 2> gpurun_out/r5/bandps/mid.err || { echo "sweep failed"; tail -5 gpurun_out/r5/bandps/mid.err; exit 1; }
cat gpurun_out/r5/bandps/mid.jsonl
