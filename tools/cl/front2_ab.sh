# A/B: the pipelined frame's front passes (G-buffer, PT_1, temporal) as 2 sequences (back: 2 by default)
set -o pipefail
AB=$'PTX_AB=\nPTX_AB=PIPE_STREAMS=2' REPS=2 TAG=ab_front2 bash tools/ab_env.sh || exit 1
