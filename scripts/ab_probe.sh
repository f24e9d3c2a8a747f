# A/B timing of library builds on one box: GPD_LIB=<lib> GPD_WT=<w> bench.py (sweep included).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
P=gym_pybullet_drones_routing_amd
i=0
for cfg in ${AB_CFGS:-"old 3" "new 3" "old 3" "new 3"}; do
  set -- $cfg
  lib=$P/libgpd.so; [ $1 = old ] && lib=$P/libgpd_old.so
  i=$((i+1))
  GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$lib GPD_WT=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/ab/run${i}_$1_$2.json 2> gpurun_out/ab/run${i}_$1_$2.err || exit $?
done
echo done
