# round 5: kernel trace of the moving-camera headline at the current build (timeline + stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5/camprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/motion -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-configs3 --camera-path --steps 10 --warmup 3 > $O/motion.log 2>&1 || { echo "motion prof failed"; tail -5 $O/motion.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/static -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-configs3 --steps 10 --warmup 3 > $O/static.log 2>&1 || { echo "static prof failed"; tail -5 $O/static.log; exit 1; }
echo done
