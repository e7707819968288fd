# round 5: GI segments scaled with the frame (1536 px at 1080p): GI / band / loopback GPU tests,
# a finer GI segment sweep, the moving GI camera at the new default
set -o pipefail
O=gpurun_out/r5/giseg
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_gi.py tests/test_gpu_bands.py tests/test_gpu_loopback.py -m gpu -q --maxfail 3 --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "GI tests failed"; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1280
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1792
PTX_LIB_PATH=$L PTX_AB=SEG_PX=768" REPS=2 TAG=r5/giseg/ab BENCH_ARGS="--workload gi --no-configs3" bash tools/ab_env.sh || exit 1
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=SEG_PX=768" TAG=r5/giseg/cam BENCH_ARGS="--workload gi --no-configs3 --camera-path" bash tools/ab_env.sh || exit 1
echo done
