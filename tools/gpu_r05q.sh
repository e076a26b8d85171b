# round-5: LDS-DMA look-ahead in the f32 record walk -- GPU tests, then C3 / C5 f32 A/B at half spp + headline
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r05q.log 2>&1 || { tail -30 $OUT/pytest_gpu_r05q.log; exit 1; }
tail -2 $OUT/pytest_gpu_r05q.log
run() {
  if [ $1 = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$1/librtw.so; fi
  timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $2 --spp-scale 0.5 --steps 2 ${3:+--tuning $3} \
    2>> $OUT/ab_r05q.err | sed "s/^{/{\"variant\": \"$1\", /" >> $OUT/ab_r05q.jsonl || exit $?
}
for round in 1 2; do
  run tree f32; run nodma f32
  echo "round $round done"
done
unset RTW_LIB_OVERRIDE
timeout -k 10 300 python tools/ab_bench.py --variants tree --modes f64,f32 --rounds 1 > $OUT/ab_head_r05q.jsonl 2> $OUT/ab_head_r05q.err || exit $?
