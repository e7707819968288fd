# launch-shape knobs re-checked after the frame-chain changes (folded light segments, temporal
# split): back sequences 1 / 2, pixel segments 768 / 1536, same box, 2 reps
set -o pipefail
AB=$'PTX_AB=\nPTX_AB=PIPE_BACK_STREAMS=1\nPTX_AB=SEG_PX=768\nPTX_AB=SEG_PX=1536' REPS=2 TAG=ab_retune BENCH_ARGS="--no-configs3" bash tools/ab_env.sh || exit 1
