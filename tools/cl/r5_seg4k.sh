# round 5 (late): the one-GPU 4K frame (configs[3] on one handle) at 4096 / 6144 / 7168-pixel segments
set -o pipefail
O=gpurun_out/r5/seg4k
mkdir -p $O
L=$PWD/pathtracerdemo_amd/libptx_ab.so
i=0
for rep in 1 2; do
  for v in "" SEG_PX=6144 SEG_PX=7168; do
    i=$((i+1))
    PTX_LIB_PATH=$L PTX_AB=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/run_$i.log 2>&1 || { echo "bench failed"; tail -5 $O/run_$i.log; exit 1; }
    tail -1 $O/run_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('configs3_one_gpu') or {}; print('rep $rep [$v]', d['value'], 'c3_4k', c.get('value'))"
  done
done
