# A/B of two library builds (libgpd_old.so vs libgpd.so) on bench.py's other BASELINE configs
# (config 3, config 4, the controller and PYB cases), alternating builds on one box.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab_cfg
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
i=0
for which in ${AB_LIBS:-old new old new}; do
  i=$((i+1))
  lib=$P/libgpd.so; [ $which = old ] && lib=$P/libgpd_old.so
  GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$lib timeout -k 10 300 python -c "
import json, torch, bench
print(json.dumps(bench.other_configs(torch.device('cuda:0'), 'f64', 'rpm')))" > $OUT/run${i}_$which.json 2> $OUT/run${i}_$which.err || exit $?
done
echo done
