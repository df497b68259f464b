# Round 6: where config 2's sweep writes go (gs_sweep_kernel<12,2,16,4>, init regime):
# WRITE_SIZE / FETCH_SIZE passes (separate rocprofv3 runs, kernel trace only) of the
# shipped build and of the attribution builds without the aggregate flush
# (-DGS_DIAG_NOFLUSH) and without the result stores (-DGS_DIAG_NOOUT).  Each build is
# copied over libgibbs_hip.so of this box's scratch copy for its passes, then restored.
set -o pipefail
OUT=gpurun_out/${TAG:-r6writes}
mkdir -p $OUT
D=gibbssampling_amd
cp $D/libgibbs_hip.so $OUT/../shipped_lib.so
for v in shipped noflush noout; do
  if [ $v = shipped ]; then cp $OUT/../shipped_lib.so $D/libgibbs_hip.so; else cp $D/libgibbs_hip_$v.so $D/libgibbs_hip.so; fi
  mkdir -p $OUT/$v
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $OUT/$v/$c -o run --output-format csv -- python3 tools/regime_bench.py --configs cfg2 --regimes init --steps 10 --warmup 2 > $OUT/$v/$c.log 2>&1 || { cp $OUT/../shipped_lib.so $D/libgibbs_hip.so; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/$v gs_sweep_kernel > $OUT/$v/summary.txt
done
cp $OUT/../shipped_lib.so $D/libgibbs_hip.so
rm -f $OUT/../shipped_lib.so
for v in shipped noflush noout; do echo "== $v"; cat $OUT/$v/summary.txt; done
