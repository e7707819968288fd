# round 4 final build: GPU suite + smoke, then the headline's evidence (rocprofv3 + PMC + bench line)
set -o pipefail
bash tools/cl/r4_suite.sh || exit 1
WLS=reuse bash tools/cl/evidence_r4.sh
