# round 5: configs[3] bands at the streamed trace walk -- the r4 cut re-timed alone with the
# exchange's one-GPU proxy (110 us, measurement build), two measured re-cuts, the 4K one-GPU frame
set -o pipefail
mkdir -p gpurun_out/r5/bands
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
B='[[0, 555], [555, 735], [735, 886], [886, 1064], [1064, 1287], [1287, 1545], [1545, 1782], [1782, 2160]]'
PTX_AB=HALO_PROXY_US=110 timeout -k 10 600 python -u tools/band_alone.py --world 8 --bands "$B" --recut 2 > gpurun_out/r5/bands/recut_proxy110.jsonl 2> gpurun_out/r5/bands/recut.err || { echo "recut failed"; tail -5 gpurun_out/r5/bands/recut.err; exit 1; }
cut -c1-400 gpurun_out/r5/bands/recut_proxy110.jsonl
unset PTX_LIB_PATH
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
import bench, json
from pathtracerdemo_amd.scene.world import compile_scene
cs = compile_scene('c3_interior_32')
print(json.dumps(bench.one_gpu_rate(cs, 3840, 2160, 'reuse', 0, 10, 3)))" > gpurun_out/r5/bands/one_gpu_4k.json || { echo "4k failed"; exit 1; }
cat gpurun_out/r5/bands/one_gpu_4k.json
