# round 4: same-box A/B of library builds on the headline (bench.py --no-cpu-baseline):
# old = the round-start build (5f695e9, no pools), alt = PTX_ROOT_DEAL=0, cur = default build,
# alt_nopool = alt with PTX_AB=RESTART_POOL=0.  3 reps, interleaved.
set -o pipefail
P=$PWD/pathtracerdemo_amd
for rep in 1 2 3; do
  for v in old alt cur alt_nopool; do
    case $v in
      old) lib=$P/libptx_old.so; ab="";;
      alt) lib=$P/libptx_alt.so; ab="";;
      cur) lib=""; ab="";;
      alt_nopool) lib=$P/libptx_alt.so; ab="RESTART_POOL=0";;
    esac
    PTX_AB=$ab PTX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs3 > gpurun_out/r4_libs_$v.$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r4_libs_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])" gpurun_out/r4_libs_$v.$rep.log $v
  done
done
