# frame pipelining at 3840x2160 on one GPU (configs[3]'s frame): the 4 Mpx cap vs pipelined, and
# pipelined with 4 trace waves per SIMD
set -o pipefail
AB=$'PTX_AB=\nPTX_AB=PIPE_MAX_KPX=16384\nPTX_AB=PIPE_MAX_KPX=16384,TRACE_OCC=4' REPS=2 TAG=ab_pipe4k BENCH_ARGS="--frame 3840x2160 --no-configs3" bash tools/ab_env.sh || exit 1
