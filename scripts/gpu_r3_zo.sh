# Round 3: PYB step time against the block geometry (drones per 64-lane block): fewer drones per
# wave put fewer other drones' long contact solves on a wave's path.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zo}
mkdir -p $OUT
for rep in 1 2; do
  for dpb in 0 8 4 2; do
    echo "== dpb $dpb rep $rep" >> $OUT/dpb.log
    GPD_PROBE_DPB=$dpb timeout -k 10 200 python -u scripts/contact_probe.py fly crash rest multi2pyb 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/dpb.log || exit $?
  done
done
echo ALLDONE
