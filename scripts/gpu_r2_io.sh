# io-wave change: parity tests that run the three-wave kernel, launch-geometry timing, phase stamps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-io}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fullsize.py tests/test_gpu_boundaries.py tests/test_gpu_dist.py -m gpu -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GEOM_CASES="4096,16,3 4096,16,2 2048,16,3 8192,32,3 8192,32,2 16384,16,3 16384,64,2" ROUNDS=2 timeout -k 10 300 python -u scripts/geom_probe.py > $OUT/geom.txt 2>&1 || exit $?
STAMP_WAVES=3 STAMP_PRECS=f64 STAMP_ENVS="4096" timeout -k 10 300 python scripts/stamp_probe.py > $OUT/stamps.txt 2>&1 || exit $?
echo ALLDONE
