# straggler queries of the headline frame (diagnostic build): tools/stragglers.py
set -o pipefail
PTX_AB=WGT PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_wgt.so timeout -k 10 300 python -u tools/stragglers.py --out gpurun_out/r4_stragglers.npz > gpurun_out/r4_stragglers.txt 2>&1 || { echo "failed"; tail -20 gpurun_out/r4_stragglers.txt; exit 1; }
cat gpurun_out/r4_stragglers.txt
