set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/grid
for seg in 256 512 768; do for k in 1 3; do for st in 3; do
 PTX_SEG_PX=$seg PTX_TRACE_SPLIT=$k PTX_WAVE_STREAMS=$st timeout -k 10 200 python tools/band_timing.py --world 8 --steps 6 > gpurun_out/grid/bt_${seg}_${k}_${st}.json || exit 1
done; done; done
for st in 1 2; do PTX_SEG_PX=512 PTX_TRACE_SPLIT=1 PTX_WAVE_STREAMS=$st timeout -k 10 200 python tools/band_timing.py --world 8 --steps 6 > gpurun_out/grid/bt_512_1_${st}.json || exit 1; done
python - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/grid/*.json")):
    d=json.load(open(f)); ms=d["band_ms_alone"]
    print(f.split("/")[-1], "max %.2f mean %.2f sum %.1f one %.2f speedup %.2f" % (max(ms), sum(ms)/len(ms), sum(ms), d["one_gpu_frame_ms"], d["implied_speedup_no_comm"]))
P
