for e in "DIAG_TAG=prior" "DIAG_TAG=prior_perframe PER_FRAME=1" "DIAG_TAG=prior_fill0 PTX_DEBUG_FILL=0" "DIAG_TAG=noprior_fill255 PRIOR=0 PTX_DEBUG_FILL=255" "DIAG_TAG=noprior_fill255_nopipe PRIOR=0 PTX_DEBUG_FILL=255 PTX_PIPELINE_FRAMES=0" "DIAG_TAG=noprior_fill255_perframe PRIOR=0 PTX_DEBUG_FILL=255 PER_FRAME=1"; do
  env $e timeout -k 10 200 python -u tools/cl/reuse_second_handle_diag.py >> gpurun_out/reuse_second_handle_diag.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 gpurun_out/reuse_second_handle_diag.log; exit $rc; }
done
grep "tag=" gpurun_out/reuse_second_handle_diag.log
