# launch shape of a 1 Mpx band (configs[3]'s 8 re-cut bands, each alone in its own process):
# segment size, back sequences, frames in flight
set -o pipefail
BANDS='[[0, 568], [568, 743], [743, 880], [880, 1039], [1039, 1255], [1255, 1504], [1504, 1754], [1754, 2160]]'
for ab in "" "SEG_PX=512" "SEG_PX=768" "PIPE_BACK_STREAMS=1" "PIPE_BACK_STREAMS=3" "PIPE_DEPTH=3"; do
  PTX_AB="$ab" timeout -k 10 300 python -u tools/band_alone.py --world 8 --bands "$BANDS" > gpurun_out/bsweep.log 2>&1 || { echo "[$ab] failed"; tail -5 gpurun_out/bsweep.log; exit 1; }
  echo "[$ab] $(tail -n 1 gpurun_out/bsweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(max(d["band_ms"]), d["sum_ms"], d["band_ms"])')"
done
