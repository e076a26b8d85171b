# round-5: C3 / C5 at half spp -- next-cell prefetch variant and light-grid densities (cell records)
set -u
OUT=gpurun_out; mkdir -p $OUT
run() {  # variant precision tuning
  if [ $1 = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$1/librtw.so; fi
  timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $2 --spp-scale 0.5 --steps 2 ${3:+--tuning $3} \
    2>> $OUT/ab_r05n.err | sed "s/^{/{\"variant\": \"$1\", /" >> $OUT/ab_r05n.jsonl || exit $?
}
for round in 1 2; do
  run tree f32; run pf f32; run tree f32 light_grid=12; run tree f32 light_grid=16; run tree f32 light_grid=6
  run tree f64; run tree f64 light_grid=12
  echo "round $round done"
done
