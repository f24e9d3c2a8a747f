# Round 3: contact solve A/B, row constants in VGPRs (base) vs in LDS (ldsc), alternated.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3p}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2; do
  for v in ${AB_VARIANTS:-ldsc_base ldsc}; do
    echo "== $v rep $rep" >> $OUT/contact.log
    GPD_LIB=$P/libgpd_$v.so timeout -k 10 300 python -u scripts/contact_probe.py crash rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/contact.log || exit $?
  done
done
echo ALLDONE
