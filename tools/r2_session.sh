#!/usr/bin/env bash
# Round-2 GPU session: selected tests (PYTEST_SEL), then optionally the full -m gpu suite and
# bench lines (BENCH=1, BENCH2=1 for a 2-rank gloo rehearsal on one GPU).  Stops at the first
# crash / time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r2}
mkdir -p $OUT
if [ -n "${PYTEST_SEL:-}" ]; then
  timeout -k 10 ${SEL_TIMEOUT:-400} python -u -m pytest $PYTEST_SEL -m gpu -x -v -p timeout --timeout 240 --timeout-method thread > $OUT/sel.log 2>&1
  rc=$?; echo "selected tests rc=$rc"; tail -n 15 $OUT/sel.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${FULL:-0}" = "1" ]; then
  timeout -k 10 ${FULL_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q -p timeout --timeout 240 --timeout-method thread > $OUT/full.log 2>&1
  rc=$?; echo "full gpu suite rc=$rc"; tail -n 8 $OUT/full.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 1500 $OUT/bench.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH2:-0}" = "1" ]; then
  PTX_FORCE_DEVICE=0 PTX_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --halo torch > $OUT/bench2.log 2>&1
  rc=$?; echo "bench2 rc=$rc"; tail -c 1500 $OUT/bench2.log
  [ $rc -ne 0 ] && exit $rc
fi
exit 0
