# A/B timing of several library builds on one box, interleaved twice:
#   AB_LIBS="old v_peel ..." bash scripts/ab_libs.sh    (lib<name>.so in the package dir)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
P=gym_pybullet_drones_routing_amd
for rep in 1 2; do
  for name in $AB_LIBS; do
    lib=$P/lib$name.so; [ $name = old ] && lib=$P/libgpd_old.so; [ $name = new ] && lib=$P/libgpd.so
    GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/ab/${name}_r$rep.json 2> gpurun_out/ab/${name}_r$rep.err || exit $?
  done
done
echo done
