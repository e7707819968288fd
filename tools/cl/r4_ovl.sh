# round 4: the overlapped band spatial pass (only the start kernel per tile set, each launch sequence's
# trace rounds one launch over its adjacent slot ranges) -- band tests, then the re-cut bands with the proxy
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_bands.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_ovl_tests.log 2>&1 \
    || { echo "band tests failed"; tail -40 gpurun_out/r4_ovl_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_ovl_tests.log | tail -1
mkdir -p gpurun_out/r4_bands
B='[[0, 555], [555, 735], [735, 886], [886, 1064], [1064, 1287], [1287, 1545], [1545, 1782], [1782, 2160]]'
PTX_AB=HALO_PROXY_US=110 timeout -k 10 300 python -u tools/band_alone.py --world 8 --bands "$B" --overlap > gpurun_out/r4_bands/recut_proxy110_overlap3.jsonl 2> gpurun_out/r4_bands/ovl.err || { echo "overlap failed"; tail -5 gpurun_out/r4_bands/ovl.err; exit 1; }
tail -n 1 gpurun_out/r4_bands/recut_proxy110_overlap3.jsonl | cut -c1-400
PTX_AB=HALO_PROXY_US=110 timeout -k 10 300 python -u tools/band_alone.py --world 8 --bands "$B" > gpurun_out/r4_bands/recut_proxy110_c.jsonl 2> gpurun_out/r4_bands/nov.err || { echo "no-overlap failed"; tail -5 gpurun_out/r4_bands/nov.err; exit 1; }
tail -n 1 gpurun_out/r4_bands/recut_proxy110_c.jsonl | cut -c1-400
