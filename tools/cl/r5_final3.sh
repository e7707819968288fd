# round 5 (last): reuse on static slots at 1024-px segments -- GPU suite, smoke, reuse evidence, the
# default bench line (with the one-GPU 4K frame) and the moving camera
set -o pipefail
O=gpurun_out/r5/final3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 300 --timeout-method thread > $O/suite.log 2>&1 \
    || { echo "GPU suite failed"; tail -60 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
ROUND=r5 WORKLOADS="reuse" bash tools/round_evidence.sh || exit 1
timeout -k 10 400 python -u bench.py > $O/headline.log 2>&1 || { echo "bench failed"; tail -20 $O/headline.log; exit 1; }
tail -1 $O/headline.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('configs3_one_gpu') or {}; print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'], 'c3_4k', c.get('value'), d.get('parity', {}).get('bit_exact'))"
timeout -k 10 400 python -u bench.py --camera-path --no-configs3 > $O/camera_path.log 2>&1 || { echo "cam bench failed"; tail -20 $O/camera_path.log; exit 1; }
tail -1 $O/camera_path.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('camera', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity', {}).get('bit_exact'))"
