# per-band time alone at the re-cut bands: trace waves 4 (default below 4 Mpx) vs 5, segments 1024 vs 768
set -o pipefail
for AB in "" "TRACE_OCC=5" "SEG_PX=768" "TRACE_OCC=5,SEG_PX=768"; do
  PTX_AB=$AB timeout -k 10 200 python -u tools/band_alone.py --world 8 --bands '[[0, 579], [579, 753], [753, 893], [893, 1064], [1064, 1279], [1279, 1521], [1521, 1758], [1758, 2160]]' > gpurun_out/bo.log 2>&1 || { echo "failed $AB"; tail -5 gpurun_out/bo.log; exit 1; }
  echo "[$AB] $(tail -1 gpurun_out/bo.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(max(d["band_ms"]), d["sum_ms"])')"
done
