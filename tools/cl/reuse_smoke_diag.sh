for e in "DIAG_TAG=default" "DIAG_TAG=nopipe PTX_PIPELINE_FRAMES=0" "DIAG_TAG=nodyn PTX_TRACE_DYN=0" "DIAG_TAG=1stream PTX_PIPELINE_FRAMES=0 PTX_WAVE_STREAMS=1"; do
  env $e timeout -k 10 200 python -u tools/cl/reuse_smoke_diag.py >> gpurun_out/reuse_smoke_diag.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 gpurun_out/reuse_smoke_diag.log; exit $rc; }
done
grep "x" gpurun_out/reuse_smoke_diag.log | grep env=
