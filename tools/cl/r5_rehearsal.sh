# round 5: bench.py --gpus 2 rehearsal on a one-GPU box (gloo + host halo, both ranks on GPU 0)
set -o pipefail
PTX_DIST_BACKEND=gloo PTX_FORCE_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 --halo torch --steps 3 --warmup 1 > gpurun_out/r5_rehearsal_gloo.log 2>&1
rc=$?; echo "gloo rc=$rc: $(grep '^{' gpurun_out/r5_rehearsal_gloo.log | tail -n 1 | cut -c1-400)"
[ $rc -ne 0 ] && { tail -20 gpurun_out/r5_rehearsal_gloo.log; exit $rc; }
exit 0
