# round 4, last build (early leaf phases): the re-cut configs[3] bands of profiles/r4/bands
# (inline: profiles/r* does not travel) each timed alone, without and with the exchange's one-GPU
# proxy, and the one-GPU 4K frame for the implied speedup
set -o pipefail
mkdir -p gpurun_out/r4_bands3
B='[[0, 555], [555, 735], [735, 886], [886, 1064], [1064, 1287], [1287, 1545], [1545, 1782], [1782, 2160]]'
timeout -k 10 400 python -u tools/band_alone.py --world 8 --bands "$B" > gpurun_out/r4_bands3/alone.jsonl 2> gpurun_out/r4_bands3/alone.err || { echo "alone failed"; tail -5 gpurun_out/r4_bands3/alone.err; exit 1; }
tail -n 1 gpurun_out/r4_bands3/alone.jsonl | cut -c1-400
PTX_AB=HALO_PROXY_US=110 timeout -k 10 400 python -u tools/band_alone.py --world 8 --bands "$B" > gpurun_out/r4_bands3/proxy110.jsonl 2> gpurun_out/r4_bands3/proxy110.err || { echo "proxy failed"; tail -5 gpurun_out/r4_bands3/proxy110.err; exit 1; }
tail -n 1 gpurun_out/r4_bands3/proxy110.jsonl | cut -c1-400
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
import bench, json
from pathtracerdemo_amd.scene.world import compile_scene
cs = compile_scene('c3_interior_32')
print(json.dumps(bench.one_gpu_rate(cs, 3840, 2160, 'reuse', 0, 10, 3)))" > gpurun_out/r4_bands3/one_gpu_4k.json || { echo "4k failed"; exit 1; }
cat gpurun_out/r4_bands3/one_gpu_4k.json
