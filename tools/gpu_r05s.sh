# round-5: f64 walk on the shared list-order template -- GPU tests, C3 / C5 f64 vs the committed tree; f32 piece sizes
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r05s.log 2>&1 || { tail -30 $OUT/pytest_gpu_r05s.log; exit 1; }
tail -2 $OUT/pytest_gpu_r05s.log
run() {
  if [ $1 = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$1/librtw.so; fi
  timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $2 --spp-scale 0.5 --steps 2 ${3:+--tuning $3} \
    2>> $OUT/ab_r05s.err | sed "s/^{/{\"variant\": \"$1\", /" >> $OUT/ab_r05s.jsonl || exit $?
}
for round in 1 2; do
  run tree f64; run head f64
  run tree f32; run tree f32 grid_piece=6; run tree f32 grid_piece=8; run tree f32 grid_piece=16
  echo "round $round done"
done
