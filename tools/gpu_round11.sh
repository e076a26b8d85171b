set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > $OUT/pytest_gpu_r01_v11.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu_r01_v11.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $OUT/bench_r01_v11.json 2> $OUT/bench_r01_v11.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench_r01_v11.json; tail -2 $OUT/bench_r01_v11.err
[ $rc -eq 0 ] || exit $rc
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU" bash tools/profile.sh r01_v11 --steps 2 --warmup 1 --no-cpu-baseline
