# trace occupancy / segment size A/B after the flattened instance loop (1080p C3 reuse; 4K one GPU)
set -o pipefail
AB=$'PTX_AB=\nPTX_AB=TRACE_OCC=5\nPTX_AB=SEG_PX=512\nPTX_AB=SEG_PX=1024' REPS=2 TAG=ab_occ bash tools/ab_env.sh || exit 1
AB=$'PTX_AB=\nPTX_AB=TRACE_OCC=4' REPS=2 TAG=ab_occ4k BENCH_ARGS="--width 3840 --height 2160 --steps 8" bash tools/ab_env.sh || exit 1
