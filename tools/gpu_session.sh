#!/usr/bin/env bash
# One gpurun session: GPU parity tests, then a short bench. Stops on any crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 ${TEST_TIMEOUT:-420} python -u -m pytest tests -m gpu -q -s -p timeout --timeout 150 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest crashed/timed out"; exit $rc; fi
if [ "${NO_BENCH:-0}" = "1" ]; then exit 0; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -n 5 gpurun_out/bench.log
exit $rc
