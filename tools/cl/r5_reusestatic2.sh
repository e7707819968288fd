# round 5: the headline's whole-image frames on static slots at ~1150 segments (REUSE_STATIC) --
# GPU suite, then A/B against dynamic batches at 1024 px, 1080p and the one-GPU 4K frame, still and moving
set -o pipefail
O=gpurun_out/r5/reusestatic2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -60 $O/suite.log; exit 1; }
tail -1 $O/suite.log
L=$PWD/pathtracerdemo_amd/libptx_ab.so
i=0
for rep in 1 2; do
  for v in 1 0; do
    i=$((i+1))
    PTX_LIB_PATH=$L PTX_AB=REUSE_STATIC=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/run_$i.log 2>&1 || { echo "bench failed"; tail -5 $O/run_$i.log; exit 1; }
    tail -1 $O/run_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('configs3_one_gpu') or {}; print('rep $rep REUSE_STATIC=$v', d['value'], d['ms_per_step'], d['roofline']['frac'], 'c3_4k', c.get('value'))"
  done
done
for v in 1 0; do
  PTX_LIB_PATH=$L PTX_AB=REUSE_STATIC=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs3 --camera-path > $O/cam_$v.log 2>&1 || { echo "cam bench failed"; tail -5 $O/cam_$v.log; exit 1; }
  tail -1 $O/cam_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cam REUSE_STATIC=$v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
echo done
