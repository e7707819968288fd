# A/B: the pipelined frame's spatial + PT_4 as 2 / 3 launch sequences (1 = default)
set -o pipefail
AB=$'PTX_AB=\nPTX_AB=PIPE_BACK_STREAMS=2\nPTX_AB=PIPE_BACK_STREAMS=3' REPS=2 TAG=ab_back bash tools/ab_env.sh || exit 1
