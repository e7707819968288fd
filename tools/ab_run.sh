#!/usr/bin/env bash
# Parity subset (TESTS) on the default library, then an env A/B (AB: newline-separated lines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-abr}
mkdir -p gpurun_out/$TAG
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest $TESTS -m gpu -x -q -p timeout --timeout 200 --timeout-method thread > gpurun_out/$TAG/parity.log 2>&1
  rc=$?; echo "parity rc=$rc"; tail -n 3 gpurun_out/$TAG/parity.log; [ $rc -ne 0 ] && exit $rc
fi
[ -n "${AB:-}" ] && AB="$AB" TAG=$TAG bash tools/ab_env.sh
exit 0
