# round 4: the re-cut configs[3] bands (profiles/r4/bands/band_alone_recut3.jsonl) with the
# exchange's one-GPU proxy and the halo overlap (interior spatial rows while the halo is in flight)
set -o pipefail
mkdir -p gpurun_out/r4_bands
B=$(python3 -c "import json; print(json.dumps(json.loads(open('profiles/r4/bands/band_alone_recut3.jsonl').read().strip().splitlines()[-1])['bands']))")
PTX_AB=HALO_PROXY_US=110 timeout -k 10 300 python -u tools/band_alone.py --world 8 --bands "$B" --overlap > gpurun_out/r4_bands/proxy110_overlap.jsonl 2> gpurun_out/r4_bands/proxy110_overlap.err || { echo "proxy overlap failed"; tail -5 gpurun_out/r4_bands/proxy110_overlap.err; exit 1; }
tail -n 1 gpurun_out/r4_bands/proxy110_overlap.jsonl | cut -c1-400
timeout -k 10 300 python -u tools/band_alone.py --world 8 --bands "$B" --overlap > gpurun_out/r4_bands/overlap.jsonl 2> gpurun_out/r4_bands/overlap.err || { echo "overlap failed"; tail -5 gpurun_out/r4_bands/overlap.err; exit 1; }
tail -n 1 gpurun_out/r4_bands/overlap.jsonl | cut -c1-400
PTX_AB=HALO_PROXY_US=110 timeout -k 10 300 python -u tools/band_alone.py --world 8 --bands "$B" > gpurun_out/r4_bands/proxy110_b.jsonl 2> gpurun_out/r4_bands/proxy110_b.err || { echo "proxy failed"; tail -5 gpurun_out/r4_bands/proxy110_b.err; exit 1; }
tail -n 1 gpurun_out/r4_bands/proxy110_b.jsonl | cut -c1-400
