# segment size by frame size: 1 Mpx bands (256 / 512), 1080p and configs[3]'s 4K one-GPU frame
# (512 / 768 / 1536 / 2048 vs 1024)
set -o pipefail
BANDS='[[0, 568], [568, 743], [743, 880], [880, 1039], [1039, 1255], [1255, 1504], [1504, 1754], [1754, 2160]]'
for ab in "SEG_PX=256" "SEG_PX=512"; do
  PTX_AB="$ab" timeout -k 10 300 python -u tools/band_alone.py --world 8 --bands "$BANDS" > gpurun_out/bsweep2.log 2>&1 || { echo "[$ab] failed"; tail -5 gpurun_out/bsweep2.log; exit 1; }
  echo "[$ab] $(tail -n 1 gpurun_out/bsweep2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(max(d["band_ms"]), d["sum_ms"], d["band_ms"])')"
done
for ab in "" "SEG_PX=512" "SEG_PX=768" "SEG_PX=1536" "SEG_PX=2048"; do
  PTX_AB="$ab" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/seg2.log 2>&1 || { echo "[$ab] bench failed"; tail -5 gpurun_out/seg2.log; exit 1; }
  echo "[$ab] $(grep '^{' gpurun_out/seg2.log | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["configs3_one_gpu"]["value"])')"
done
