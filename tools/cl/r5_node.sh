# round 5: the Node engine loop (NativeRenderer) with ReSTIR GI added
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_node_engine.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r5_node.log 2>&1 || { echo "node tests failed"; tail -40 gpurun_out/r5_node.log; exit 1; }
tail -5 gpurun_out/r5_node.log
