# round-5: f32 light-grid kernels -- list-order walk with per-trip pieces (f32list) and 3 waves per SIMD (…3)
set -u
OUT=gpurun_out; mkdir -p $OUT
run() {
  if [ $1 = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$1/librtw.so; fi
  timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $2 --spp-scale 0.5 --steps 2 ${3:+--tuning $3} \
    2>> $OUT/ab_r05t.err | sed "s/^{/{\"variant\": \"$1\", /" >> $OUT/ab_r05t.jsonl || exit $?
}
for round in 1 2; do
  for v in tree tree3 f32list f32list3; do run $v f32; done
  echo "round $round done"
done
