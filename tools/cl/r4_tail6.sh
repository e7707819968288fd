# round 4: launch tails at the round's kernels, with the neighbourhood predictor what-if
set -o pipefail
PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so timeout -k 10 300 python -u tools/trace_tail.py --frames 3 --out gpurun_out/r4_trace_tail6.json > gpurun_out/r4_trace_tail6.txt 2>&1 || { echo "tail failed"; tail -20 gpurun_out/r4_trace_tail6.txt; exit 1; }
grep -E "longest-first|^launch|^[0-9]\\.[0-9]" gpurun_out/r4_trace_tail6.txt | head -30
