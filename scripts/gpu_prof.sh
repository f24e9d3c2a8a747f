cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_r1
mkdir -p $OUT
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench -o bench --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep > $OUT/bench_stdout.json 2> $OUT/bench_stderr.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/big64 -o big64 --output-format csv -- python3 scripts/prof_step.py --envs 1048576 --precision f64 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/big32 -o big32 --output-format csv -- python3 scripts/prof_step.py --envs 1048576 --precision f32 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o fetch --output-format csv -- python3 scripts/prof_step.py --envs 1048576 --precision f64 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o write --output-format csv -- python3 scripts/prof_step.py --envs 1048576 --precision f64 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc_sq -o sq --output-format csv -- python3 scripts/prof_step.py --envs 1048576 --precision f64 > /dev/null 2>&1
echo ALLDONE
