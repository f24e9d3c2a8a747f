cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/abc
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2; do
  for v in $AB_VARIANTS; do
    echo "== $v rep $rep" >> $OUT/ab.log
    GPD_LIB=$P/libgpd_$v.so timeout -k 10 200 python -u scripts/contact_probe.py 2>&1 | grep -v amdgpu >> $OUT/ab.log || exit $?
  done
done
echo ALLDONE
