# Round 3: s_setprio for the io kernel's pose / rate waves (libgpd_prio.so) vs none (libgpd.so),
# 4096- and 1024-env step time alternated (tail_probe.py).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zp}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2 3 4; do
  for v in gpd gpd_prio; do
    GPD_LIB=$P/lib$v.so timeout -k 10 120 python -u scripts/tail_probe.py $v >> $OUT/ab.log 2>&1 || exit $?
    GPD_PROBE_ENVS=1024 GPD_LIB=$P/lib$v.so timeout -k 10 120 python -u scripts/tail_probe.py $v >> $OUT/ab.log 2>&1 || exit $?
  done
done
echo ALLDONE
