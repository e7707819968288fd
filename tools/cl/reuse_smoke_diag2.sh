for e in "DIAG_TAG=default" "DIAG_TAG=noprior PRIOR=0" "DIAG_TAG=nopipe PTX_PIPELINE_FRAMES=0"; do
  env $e timeout -k 10 200 python -u tools/cl/reuse_smoke_diag2.py >> gpurun_out/reuse_smoke_diag2.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 gpurun_out/reuse_smoke_diag2.log; exit $rc; }
done
grep "prior=" gpurun_out/reuse_smoke_diag2.log
