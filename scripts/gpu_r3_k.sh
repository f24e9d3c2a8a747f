# Round 3: bench line (raw integrator with STREAM), multi-drone PYB A/B with and without parked
# idle lanes (same box, alternated).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3k}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
# (bench leg done in r3k)
for rep in 1 2; do
  for v in nopark cur; do
    echo "== $v rep $rep" >> $OUT/contact.log
    GPD_LIB=$P/libgpd_$v.so timeout -k 10 300 python -u scripts/contact_probe.py crash rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/contact.log || exit $?
  done
done
echo ALLDONE
