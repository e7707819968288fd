# round 4: SIMD utilisation profiles, then the band vs 4K-frame kernel profiles
set -o pipefail
mkdir -p gpurun_out/r4_bandprof
bash tools/cl/r4_simd.sh || exit 1
bash tools/cl/r4_bandprof.sh
