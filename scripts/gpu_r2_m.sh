cd $GRAFT_REPO_ROOT
bash scripts/pmc_icache.sh || exit $?
AB_VARIANTS="main dma0 dma4 dma5" GEOM_CASES="4096,16,2 4096,16,3 16384,64,2 16384,64,3 65536,64,2 65536,64,3" bash scripts/ab_geom.sh || exit $?
STAMP_LIBS="stamps st_dma4 st_dma5" bash scripts/stamp_var.sh || exit $?
echo ALLDONE
