# trace-launch tails with the per-batch work breakdown (diagnostic build)
set -o pipefail
PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so timeout -k 10 300 python -u tools/trace_tail.py --frames 2 --out gpurun_out/r4_trace_tail2.json > gpurun_out/r4_trace_tail2.txt 2>&1 || { echo "tail failed"; tail -20 gpurun_out/r4_trace_tail2.txt; exit 1; }
tail -32 gpurun_out/r4_trace_tail2.txt
