# bench.py --gpus 2 rehearsals on a one-GPU box: gloo + host halo, then the RCCL path with
# both ranks on GPU 0 (RCCL may refuse two ranks on one device: that is reported, not fatal)
PTX_DIST_BACKEND=gloo PTX_FORCE_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 --halo torch --steps 3 --warmup 1 > gpurun_out/rehearsal_gloo.log 2>&1
rc=$?; echo "gloo rc=$rc: $(grep '^{' gpurun_out/rehearsal_gloo.log | tail -n 1 | cut -c1-220)"
[ $rc -gt 1 ] && { tail -20 gpurun_out/rehearsal_gloo.log; exit $rc; }
PTX_FORCE_DEVICE=0 NCCL_DEBUG=WARN timeout -k 10 180 python -u bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/rehearsal_rccl.log 2>&1
rc=$?; echo "rccl rc=$rc: $(grep '^{' gpurun_out/rehearsal_rccl.log | tail -n 1 | cut -c1-220)"
tail -8 gpurun_out/rehearsal_rccl.log
exit 0
