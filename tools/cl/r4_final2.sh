# round 4, second final build (early leaf phases): GPU suite + smoke, the headline's and C1
# ReSTIR's evidence (rocprofv3 + PMC + bench line), then the trace_core_tab K / L sweep on C1
set -o pipefail
bash tools/cl/r4_suite.sh || exit 1
WLS="reuse restir" bash tools/cl/evidence_r4.sh || exit 1
VARIANTS="g1 g2 g3 g4" REPS=2 TAG=tabk BENCH_ARGS="--workload restir" bash tools/cl/r5_multi_ab.sh
