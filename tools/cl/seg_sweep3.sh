# segment size at 4 and 8.3 Mpx: configs[3]'s frame on one GPU (1024 / 2048 / 4096, 2 reps)
# and its 2 re-cut bands (~4 Mpx each, 1024 / 2048)
set -o pipefail
for rep in 1 2; do for ab in "" "SEG_PX=2048" "SEG_PX=4096"; do
  PTX_AB="$ab" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/seg3.log 2>&1 || { echo "[$ab] bench failed"; tail -5 gpurun_out/seg3.log; exit 1; }
  echo "[$ab] $(grep '^{' gpurun_out/seg3.log | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["configs3_one_gpu"]["value"])')"
done; done
for ab in "" "SEG_PX=2048" "SEG_PX=512"; do
  PTX_AB="$ab" timeout -k 10 300 python -u tools/band_alone.py --world 2 --recut 1 > gpurun_out/bsweep3.log 2>&1 || { echo "[$ab] failed"; tail -5 gpurun_out/bsweep3.log; exit 1; }
  echo "[$ab] $(tail -n 1 gpurun_out/bsweep3.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(max(d["band_ms"]), d["sum_ms"], d["bands"], d["band_ms"])')"
done
