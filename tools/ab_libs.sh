#!/usr/bin/env bash
# Same-box A/B of library builds (PTX_LIB_PATH): optional GPU parity subset on the first
# variant (PARITY=1), then bench runs per library.  usage: LIBS="libptx.so libptx_x.so" bash tools/ab_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=$PWD/pathtracerdemo_amd
TAG=${TAG:-ablibs}
mkdir -p gpurun_out/$TAG
if [ "${PARITY:-0}" = "1" ]; then
  for L in ${PARITY_LIBS:-${LIBS%% *}}; do
    PTX_LIB_PATH=$P/$L timeout -k 10 ${PARITY_TIMEOUT:-300} python -u -m pytest ${PARITY_TESTS:-tests/test_gpu_parity.py tests/test_gpu_reuse.py} -m gpu -x -q -p timeout --timeout 120 --timeout-method thread > gpurun_out/$TAG/parity_$L.log 2>&1
    rc=$?; echo "parity $L rc=$rc"; tail -n 3 gpurun_out/$TAG/parity_$L.log
    [ $rc -ne 0 ] && exit $rc
  done
fi
AB=""
for L in $LIBS; do AB+="PTX_LIB_PATH=$P/$L ${AB_ENV:-}"$'\n'; done
AB="$AB" TAG=$TAG bash tools/ab_env.sh
