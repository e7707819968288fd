# round 5: per-kernel time of a band frame vs an eighth of the one-GPU 4K frame (rocprof, the
# production paths: pipelined 4K frame; the band alone with the proxy, measurement build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5/bandcmp
mkdir -p $O/4k $O/band
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/4k -o run --output-format csv -- \
  python3 -c "import sys; sys.path.insert(0, '$R'); import bench, json; from pathtracerdemo_amd.scene.world import compile_scene; cs = compile_scene('c3_interior_32'); print(json.dumps(bench.one_gpu_rate(cs, 3840, 2160, 'reuse', 0, 10, 3)))" > $O/4k/log.txt 2>&1 || { echo "4k failed"; tail -5 $O/4k/log.txt; exit 1; }
tail -1 $O/4k/log.txt
PTX_LIB_PATH=$R/pathtracerdemo_amd/libptx_ab.so PTX_AB=HALO_PROXY_US=110 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/band -o run --output-format csv -- \
  python3 -c "import sys; sys.path.insert(0, '$R'); import bench; from pathtracerdemo_amd.scene.world import compile_scene; cs = compile_scene('c3_interior_32'); print(bench.calibrate_band(cs, 3840, 2160, 'reuse', 0, 895, 1059, bench.PASSES['reuse'], frames=10))" > $O/band/log.txt 2>&1 || { echo "band failed"; tail -5 $O/band/log.txt; exit 1; }
tail -1 $O/band/log.txt
