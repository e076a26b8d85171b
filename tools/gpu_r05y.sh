# round-5: the f64 walk's owner pdfs dealt to the wave -- GPU tests, C3 / C5 f64 A/B at half spp
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r05y.log 2>&1 || { tail -30 $OUT/pytest_gpu_r05y.log; exit 1; }
tail -2 $OUT/pytest_gpu_r05y.log
run() {
  if [ $1 = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$1/librtw.so; fi
  timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $2 --spp-scale 0.5 --steps 2 ${3:+--tuning $3} \
    2>> $OUT/ab_r05y.err | sed "s/^{/{\"variant\": \"$1\", /" >> $OUT/ab_r05y.jsonl || exit $?
}
for round in 1 2; do
  run tree f64; run nodeal f64
  echo "round $round done"
done
