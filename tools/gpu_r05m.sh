# round-5: GPU tests on the tree, then A/B of head / norec / tree (headline f64 + f32, C3 / C5 both precisions at half spp)
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r05m.log 2>&1 || { tail -30 $OUT/pytest_gpu_r05m.log; exit 1; }
tail -2 $OUT/pytest_gpu_r05m.log
timeout -k 10 400 python tools/ab_bench.py --variants head,tree --modes f64,f32 --rounds 2 > $OUT/ab_head_r05m.jsonl 2> $OUT/ab_head_r05m.err || exit $?
for round in 1 2; do
  for v in head norec tree; do
    for p in f32 f64; do
      if [ $v = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$v/librtw.so; fi
      timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $p --spp-scale 0.5 --steps 2 \
        2>> $OUT/ab_walk_r05m.err | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/ab_walk_r05m.jsonl || exit $?
    done
    echo "round $round $v done"
  done
done
unset RTW_LIB_OVERRIDE
