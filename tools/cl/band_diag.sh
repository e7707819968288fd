for e in "X=equal" "PTX_TRACE_DYN=1" "PTX_WAVE_STREAMS=1"; do
  a=""; [ "$e" = "X=equal" ] && a="--bands equal"
  env $e timeout -k 10 300 python -u tools/band_timing.py --world 8 --steps 6 $a > gpurun_out/band_diag.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/band_diag.log; exit $rc; }
  echo "[$e] $(tail -n 1 gpurun_out/band_diag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["bands"], d["band_ms_alone"], d["one_gpu_frame_ms"], d["implied_speedup_no_comm"])')"
done
