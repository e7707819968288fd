# wavefront segment size A/B (1080p C3 reuse, GI, TEST_MCPT)
set -o pipefail
AB=$'PTX_AB=SEG_PX=768\nPTX_AB=SEG_PX=1024\nPTX_AB=SEG_PX=1536\nPTX_AB=SEG_PX=2048' REPS=2 TAG=ab_seg bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=SEG_PX=768\nPTX_AB=SEG_PX=1024\nPTX_AB=SEG_PX=1536' REPS=1 TAG=ab_seg_g BENCH_ARGS="--workload gi" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=SEG_PX=768\nPTX_AB=SEG_PX=1024\nPTX_AB=SEG_PX=1536' REPS=1 TAG=ab_seg_m BENCH_ARGS="--workload mcpt" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=SEG_PX=768\nPTX_AB=SEG_PX=1024\nPTX_AB=SEG_PX=1536' REPS=1 TAG=ab_seg_r BENCH_ARGS="--workload restir" bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=SEG_PX=768\nPTX_AB=SEG_PX=1024\nPTX_AB=SEG_PX=1536' REPS=1 TAG=ab_seg_4k BENCH_ARGS="--width 3840 --height 2160 --steps 8" bash tools/ab_env.sh || exit 1
