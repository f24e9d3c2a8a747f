# Phase stamps of stamp-build variants: STAMP_LIBS="stamps st_dma0 ..." (libgpd_<v>.so; "stamps" = libgpd_stamps.so)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-stv}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for v in $STAMP_LIBS; do
  lib=$P/libgpd_$v.so
  echo "== $v" >> $OUT/stamps.log
  for w in ${STAMP_WAVES_LIST:-3}; do
    GPD_STAMPS_LIB=$lib STAMP_WAVES=$w STAMP_PRECS=f64 STAMP_ENVS="${STAMP_ENVS:-4096}" timeout -k 10 300 python scripts/stamp_probe.py 2>/dev/null | grep -v amdgpu >> $OUT/stamps.log || exit $?
  done
done
echo ALLDONE
