# round 5: TEST_MCPT frames pipelined -- MCPT GPU tests, then launch-shape A/B (C1 1080p, measurement build)
set -o pipefail
O=gpurun_out/r5/pipemcpt
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_present.py tests/test_gpu_cull.py tests/test_gpu_large_tables.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "GPU tests failed"; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L=$PWD/pathtracerdemo_amd/libptx_ab.so
AB="PTX_LIB_PATH=$L PTX_AB=
PTX_LIB_PATH=$L PTX_AB=PIPE_MCPT=0
PTX_LIB_PATH=$L PTX_AB=TRACE_DYN=0
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536
PTX_LIB_PATH=$L PTX_AB=SEG_PX=1536,TRACE_DYN=0
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=2
PTX_LIB_PATH=$L PTX_AB=PIPE_STREAMS=2,TRACE_DYN=0" REPS=2 TAG=r5/pipemcpt/ab BENCH_ARGS="--workload mcpt --no-configs3" bash tools/ab_env.sh || exit 1
echo done
