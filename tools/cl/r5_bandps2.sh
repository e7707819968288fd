# round 5 (late): band handles back on one front launch sequence per context -- band GPU tests, the
# middle band alone with the proxy, and the 8 re-cut bands of configs[3] (recut_static_batches cut)
set -o pipefail
O=gpurun_out/r5/bandps2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_bands.py tests/test_gpu_loopback.py -m gpu -q --maxfail 3 --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "band tests failed"; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so
P=HALO_PROXY_US=110
timeout -k 10 300 python -u tools/band_knobs.py --band 895,1061 --ab "$P" "$P" > $O/mid.jsonl 2> $O/mid.err || { echo "sweep failed"; tail -5 $O/mid.err; exit 1; }
cat $O/mid.jsonl
