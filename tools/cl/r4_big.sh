# round 4: split motion pass (tests, suite, moving-camera A/B), then the configs[3] bands
set -o pipefail
bash tools/cl/r4_msplit.sh || exit 1
bash tools/cl/r4_bands.sh
