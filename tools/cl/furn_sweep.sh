# launch-shape sweep on the furnished C3 (13 instances): is a scene-dependent shape worth it?
set -o pipefail
AB=$'PTX_AB=\nPTX_AB=TRACE_OCC=5\nPTX_AB=SEG_PX=768\nPTX_AB=SEG_PX=1536\nPTX_AB=SEG_PX=2048\nPTX_AB=PIPE_BACK_STREAMS=3\nPTX_AB=PIPE_BACK_STREAMS=1\nPTX_AB=PIPE_DEPTH=3'
AB="$AB" REPS=1 TAG=furn_sweep BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=TRACE_OCC=5\nPTX_AB=SEG_PX=1536' REPS=1 TAG=furn_sweep_b BENCH_ARGS="--no-configs3 --scene c3_furnished" bash tools/ab_env.sh || exit 1
