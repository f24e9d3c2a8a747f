# Round 3: the io wave's history gathered into registers before the hand-offs (GPD_IO_GATHER=1,
# libgpd.so) vs round 2's LDS-DMA after them (libgpd_dma.so): GPU tests on the new default, then
# the 4096-env step time alternated (tail_probe.py, graph replay, median of 7 regions).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zi}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2 3 4; do
  for v in gpd gpd_dma; do
    GPD_LIB=$P/lib$v.so timeout -k 10 120 python -u scripts/tail_probe.py $v >> $OUT/ab.log 2>&1 || exit $?
    GPD_PROBE_ENVS=1024 GPD_LIB=$P/lib$v.so timeout -k 10 120 python -u scripts/tail_probe.py $v >> $OUT/ab.log 2>&1 || exit $?
  done
done
echo ALLDONE
