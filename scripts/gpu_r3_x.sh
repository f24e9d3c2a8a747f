# Round 3: the final contact solve (v2 loop, refined-reciprocal setup, parked outer values):
# bullet + golden + boundary parity, then the contact probe (3 alternations of one library).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3x}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_bullet.py tests/test_golden.py tests/test_gpu_boundaries.py tests/test_gpu_pid.py -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2 3; do
  echo "== final rep $rep" >> $OUT/probe.log
  timeout -k 10 200 python -u scripts/contact_probe.py fly crash rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/probe.log || exit $?
done
echo ALLDONE
