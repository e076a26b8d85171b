# round-5: f64 walk owners -- dealt pdfs, two 16-byte slot reads, big-list candidates once per walk
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r05aa.log 2>&1 || { tail -30 $OUT/pytest_gpu_r05aa.log; exit 1; }
tail -2 $OUT/pytest_gpu_r05aa.log
run() {
  if [ $1 = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$1/librtw.so; fi
  timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $2 --spp-scale 0.5 --steps 2 ${3:+--tuning $3} \
    2>> $OUT/ab_r05aa.err | sed "s/^{/{\"variant\": \"$1\", /" >> $OUT/ab_r05aa.jsonl || exit $?
}
for round in 1 2; do
  run tree f64; run head f64
  echo "round $round done"
done
unset RTW_LIB_OVERRIDE
timeout -k 10 200 python tools/clock_profile.py run --config C5 --precision f64 --spp 32 >> $OUT/clock_r05aa.jsonl 2>> $OUT/clock_r05aa.err || exit $?
