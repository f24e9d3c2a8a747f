# Round 3: contact setup skipping the rim points no lane of the wave touches (libgpd_skip.so)
# vs the default (libgpd.so), contact probe alternated.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zk}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2 3; do
  for v in gpd gpd_skip; do
    echo "== $v rep $rep" >> $OUT/ab.log
    GPD_LIB=$P/lib$v.so timeout -k 10 200 python -u scripts/contact_probe.py crash rest multi multi2pyb 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/ab.log || exit $?
  done
done
echo ALLDONE
