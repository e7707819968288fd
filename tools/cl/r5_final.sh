# round 5, final build: GPU suite + smoke, then every workload's bench line (static headline with
# its CPU baselines, the moving camera, GI, C1 ReSTIR, TEST_MCPT)
set -o pipefail
bash tools/cl/r5_suite.sh || exit 1
mkdir -p gpurun_out/r5/final
for a in "--camera-path --no-configs3 --no-cpu-baseline" "--workload gi --no-cpu-baseline" "--workload restir --no-cpu-baseline" "--workload mcpt --no-cpu-baseline"; do
  n=$(echo "$a" | tr -d ' -' | cut -c1-24)
  timeout -k 10 300 python3 bench.py $a > gpurun_out/r5/final/$n.log 2>&1 || { echo "bench $a failed"; tail -5 gpurun_out/r5/final/$n.log; exit 1; }
  echo "$a: $(tail -1 gpurun_out/r5/final/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"])')"
done
