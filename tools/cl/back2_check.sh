# two back sequences by default: GPU suite, headline A/B, bands alone (2 vs 1 back sequences)
set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/b2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/b2_tests.log; exit 1; }
tail -1 gpurun_out/b2_tests.log
AB=$'PTX_AB=\nPTX_AB=PIPE_BACK_STREAMS=1' REPS=2 TAG=ab_back2 bash tools/ab_env.sh || exit 1
for AB in "" "PIPE_BACK_STREAMS=1"; do
  PTX_AB=$AB timeout -k 10 200 python -u tools/band_alone.py --world 8 --bands '[[0, 579], [579, 753], [753, 893], [893, 1064], [1064, 1279], [1279, 1521], [1521, 1758], [1758, 2160]]' > gpurun_out/bo2.log 2>&1 || { echo "failed $AB"; exit 1; }
  echo "bands [$AB] $(tail -1 gpurun_out/bo2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(max(d["band_ms"]), d["sum_ms"])')"
done
