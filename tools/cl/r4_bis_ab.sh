# round 4: bisect the trace_queue regression: old = round-start build, bis = current tree with
# the round-start ptx_wave.hip (no restart pools, per-batch trace_batch), cur = current build
set -o pipefail
P=$PWD/pathtracerdemo_amd
for rep in 1 2; do
  for v in old bis cur; do
    case $v in
      old) lib=$P/libptx_old.so; ab="";;
      alt) lib=$P/libptx_alt.so; ab="";;
      cur) lib=""; ab="";;
      bis) lib=$P/libptx_bis.so; ab="";;
    esac
    PTX_AB=$ab PTX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs3 > gpurun_out/r4_libs_$v.$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r4_libs_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])" gpurun_out/r4_libs_$v.$rep.log $v
  done
done
