# bench.py --gpus N with the band calibration, ranks sharing GPU 0 over gloo (host halo)
for n in 2 8; do
  PTX_DIST_BACKEND=gloo PTX_FORCE_DEVICE=0 timeout -k 10 400 python -u bench.py --gpus $n --halo torch --steps 3 --warmup 1 > gpurun_out/calib_$n.log 2>&1
  rc=$?; echo "n=$n rc=$rc"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/calib_$n.log; exit $rc; }
  grep '^{' gpurun_out/calib_$n.log | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["bands"])'
done
