# round 5: the streamed walk's refill threshold on static slots (a band alone, proxy): 16 / 32 / 48
set -o pipefail
P=HALO_PROXY_US=110
for L in libptx_ab.so libptx_rf16.so libptx_rf48.so libptx_ab.so; do
  PTX_LIB_PATH=$PWD/pathtracerdemo_amd/$L timeout -k 10 300 python -u tools/band_knobs.py --band 895,1059 --ab "$P" | sed "s#^#$L #" || exit 1
done
LIBS="libptx_ab.so libptx_rf16.so libptx_rf48.so" REPS=1 TAG=r5/c1rf BENCH_ARGS="--no-configs3 --workload restir" bash tools/ab_libs.sh || exit 1
