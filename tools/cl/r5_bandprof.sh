# round 5: kernel trace of one configs[3] band frame timed alone (where a band's 2.5 ms go)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5/bandprof
mkdir -p $O
export PTX_LIB_PATH=$R/pathtracerdemo_amd/libptx_ab.so PTX_AB=HALO_PROXY_US=110
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
  python3 -c "import sys; sys.path.insert(0, '$R'); import bench; from pathtracerdemo_amd.scene.world import compile_scene; cs = compile_scene('c3_interior_32'); print(bench.calibrate_band(cs, 3840, 2160, 'reuse', 0, 895, 1061, bench.PASSES['reuse'], frames=10))" > $O/log.txt 2>&1 || { echo "prof failed"; tail -5 $O/log.txt; exit 1; }
tail -1 $O/log.txt
