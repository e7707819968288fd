# round 4: the motion start kernel with one job_emit site -- motion tests, then the moving-camera
# bench: cur (3 waves/SIMD), alt (2 waves), prev (three inlined job_emit sites, 2 waves)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_bands.py -x -q --timeout 240 --timeout-method thread -k "moving or motion or camera or communicator or interleaved" > gpurun_out/r4_mstart_tests.log 2>&1 \
    || { echo "motion tests failed"; tail -40 gpurun_out/r4_mstart_tests.log; exit 1; }
tail -1 gpurun_out/r4_mstart_tests.log
P=$PWD/pathtracerdemo_amd
for rep in 1 2; do
  for v in cur alt prev; do
    lib=""; [ "$v" = alt ] && lib=$P/libptx_alt.so; [ "$v" = prev ] && lib=$P/libptx_prev.so
    PTX_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --camera-path --no-cpu-baseline --no-configs3 > gpurun_out/r4_mstart_$v.$rep.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4_mstart_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r4_mstart_$v.$rep.log $v
  done
done
