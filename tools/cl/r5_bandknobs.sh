# round 5: which switches shorten a configs[3] band frame at the streamed walk (measurement
# build, 110 us exchange proxy); then the 1080p headline's segment size
set -o pipefail
mkdir -p gpurun_out/r5/bandknobs
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
P=HALO_PROXY_US=110
timeout -k 10 900 python -u tools/band_knobs.py --band 895,1061 --ab "$P" "$P,SEG_PX=256" "$P,SEG_PX=1024" "$P,PIPE_DEPTH=3" "$P,PIPE_BACK_STREAMS=1" "$P,PIPE_BACK_STREAMS=3" "$P,TRACE_DYN=0" "$P,OVERLAP_START=0" "$P" > gpurun_out/r5/bandknobs/mid.jsonl 2> gpurun_out/r5/bandknobs/mid.err || { echo "sweep failed"; tail -5 gpurun_out/r5/bandknobs/mid.err; exit 1; }
cat gpurun_out/r5/bandknobs/mid.jsonl
timeout -k 10 300 python -u tools/band_knobs.py --band 895,1061 --overlap --ab "$P" "$P,PIPE_DEPTH=3" > gpurun_out/r5/bandknobs/mid_ovl.jsonl 2>> gpurun_out/r5/bandknobs/mid.err || { echo "sweep2 failed"; exit 1; }
cat gpurun_out/r5/bandknobs/mid_ovl.jsonl
AB="PTX_LIB_PATH=$PTX_LIB_PATH"$'\n'"PTX_LIB_PATH=$PTX_LIB_PATH PTX_AB=SEG_PX=512"$'\n'"PTX_LIB_PATH=$PTX_LIB_PATH PTX_AB=SEG_PX=2048"$'\n'"PTX_LIB_PATH=$PTX_LIB_PATH PTX_AB=PIPE_DEPTH=3" \
  TAG=r5/bandknobs/hd BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
