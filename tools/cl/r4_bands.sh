# round 4: configs[3]'s 8 bands each timed alone (one process per band, as a rank runs it) with
# three measured re-cuts, then the final bands with the exchange's one-GPU proxy
# (PTX_AB=HALO_PROXY_US=110: the edge rows copied device to device + a 110 us wait standing for
# the 2 x 16.6 MB xGMI transfer) and the one-GPU 4K frame for the implied speedup
set -o pipefail
mkdir -p gpurun_out/r4_bands
timeout -k 10 900 python -u tools/band_alone.py --world 8 --recut 3 > gpurun_out/r4_bands/recut3.jsonl 2> gpurun_out/r4_bands/recut3.err || { echo "recut failed"; tail -5 gpurun_out/r4_bands/recut3.err; exit 1; }
tail -n 1 gpurun_out/r4_bands/recut3.jsonl | cut -c1-400
B=$(python3 -c "import json; print(json.dumps(json.loads(open('gpurun_out/r4_bands/recut3.jsonl').read().strip().splitlines()[-1])['bands']))")
PTX_AB=HALO_PROXY_US=110 timeout -k 10 300 python -u tools/band_alone.py --world 8 --bands "$B" > gpurun_out/r4_bands/proxy110.jsonl 2> gpurun_out/r4_bands/proxy110.err || { echo "proxy failed"; tail -5 gpurun_out/r4_bands/proxy110.err; exit 1; }
tail -n 1 gpurun_out/r4_bands/proxy110.jsonl | cut -c1-400
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
import bench, json
from pathtracerdemo_amd.scene.world import compile_scene
cs = compile_scene('c3_interior_32')
print(json.dumps(bench.one_gpu_rate(cs, 3840, 2160, 'reuse', 0, 10, 3)))" > gpurun_out/r4_bands/one_gpu_4k.json || { echo "4k failed"; exit 1; }
cat gpurun_out/r4_bands/one_gpu_4k.json
