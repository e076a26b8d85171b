# round-5: the light kernels' empty-list NaN direction as a select -- GPU tests, C3 / C5 A/B vs the committed tree
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r05ae.log 2>&1 || { tail -30 $OUT/pytest_gpu_r05ae.log; exit 1; }
tail -2 $OUT/pytest_gpu_r05ae.log
run() {
  if [ $1 = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$1/librtw.so; fi
  timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $2 --spp-scale 0.5 --steps 2 ${3:+--tuning $3} \
    2>> $OUT/ab_r05ae.err | sed "s/^{/{\"variant\": \"$1\", /" >> $OUT/ab_r05ae.jsonl || exit $?
}
run tree f64; run head f64; run tree f32; run head f32
run tree f64; run head f64
