# round 4: the motion pass's light segments finished by its combine -- motion tests (both the
# whole and the split pass), then the moving-camera bench with and without (PTX_AB=MOTION_FOLD)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_bands.py -x -v --timeout 240 --timeout-method thread -k "moving or motion or camera or communicator or interleaved" > gpurun_out/r4_mfold_tests.log 2>&1 \
    || { echo "motion tests failed"; tail -40 gpurun_out/r4_mfold_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_mfold_tests.log | tail -1
PTX_AB=MOTION_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py -x -q --timeout 240 --timeout-method thread -k "moving or camera or interleaved" > gpurun_out/r4_mfold_tests_split.log 2>&1 \
    || { echo "split motion tests failed"; tail -40 gpurun_out/r4_mfold_tests_split.log; exit 1; }
tail -1 gpurun_out/r4_mfold_tests_split.log
for rep in 1 2; do
  for ab in MOTION_FOLD=1 MOTION_FOLD=0; do
    PTX_AB=$ab timeout -k 10 300 python -u bench.py --camera-path --no-cpu-baseline --no-configs3 > gpurun_out/r4_mfold_$ab.$rep.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4_mfold_$ab.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r4_mfold_$ab.$rep.log $ab
  done
done
