# Round 3, drone <-> drone contact: the full run (scripts/gpu_r3_full.sh) on the final code, then the
# multi-drone PYB probe with and without the drone contact.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3dc2}
RUN_TAG=${RUN_TAG:-r3dc2} bash scripts/gpu_r3_full.sh || exit $?
timeout -k 10 300 python -u scripts/contact_probe.py multi2pyb multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " > $OUT/probe_dc.log || exit $?
GPD_PROBE_NODC=1 timeout -k 10 300 python -u scripts/contact_probe.py multi2pyb multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " > $OUT/probe_nodc.log || exit $?
echo ALLDONE
