# A/B of library variants (libgpd_<v>.so built by _build.build(variant=v, defines=...)) with the
# geometry probe, interleaved: AB_VARIANTS="v1 v2 ..." GEOM_CASES="E,dpb,waves ..." bash scripts/ab_geom.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-ab}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2; do
  for v in $AB_VARIANTS; do
    lib=$P/libgpd_$v.so; [ $v = main ] && lib=$P/libgpd.so
    echo "== $v rep $rep" >> $OUT/ab_geom.log
    ROUNDS=1 GPD_LIB=$lib timeout -k 10 200 python -u scripts/geom_probe.py 2>/dev/null | grep -v amdgpu >> $OUT/ab_geom.log || exit $?
  done
done
echo ALLDONE
