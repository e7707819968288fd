# smoke() under each library build (PTX_LIB_PATH); stops at anything but pass / assertion failure
P=$PWD/pathtracerdemo_amd
for L in $LIBS; do
  PTX_LIB_PATH=$P/$L timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$L.log 2>&1
  rc=$?
  echo "$L rc=$rc $(tail -n 1 gpurun_out/smoke_$L.log | cut -c1-150)"
  [ $rc -gt 1 ] && exit $rc
done
exit 0
