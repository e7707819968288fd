# round 4: the motion temporal pass split around the wait (pipelined whole-image frames) --
# motion + band tests, the GPU suite, then the moving-camera bench with and without the split
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_bands.py -x -v --timeout 240 --timeout-method thread -k "moving or motion or camera or communicator or interleaved" > gpurun_out/r4_msplit_tests.log 2>&1 \
    || { echo "motion tests failed"; tail -40 gpurun_out/r4_msplit_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_msplit_tests.log | tail -2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_msplit_suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -40 gpurun_out/r4_msplit_suite.log; exit 1; }
tail -1 gpurun_out/r4_msplit_suite.log
for rep in 1 2; do
  for ab in MOTION_SPLIT=1 MOTION_SPLIT=0; do
    PTX_AB=$ab timeout -k 10 300 python -u bench.py --camera-path --no-cpu-baseline --no-configs3 > gpurun_out/r4_msplit_$ab.$rep.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4_msplit_$ab.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r4_msplit_$ab.$rep.log $ab
  done
done
