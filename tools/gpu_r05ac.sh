# round-5: owner list length of the f64 walk (RTW_COOP64_MAX 8 / 12 / 16)
set -u
OUT=gpurun_out; mkdir -p $OUT
run() {
  if [ $1 = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$1/librtw.so; fi
  timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $2 --spp-scale 0.5 --steps 2 ${3:+--tuning $3} \
    2>> $OUT/ab_r05ac.err | sed "s/^{/{\"variant\": \"$1\", /" >> $OUT/ab_r05ac.jsonl || exit $?
}
for round in 1 2; do
  run tree f64; run max12 f64; run max16 f64
  echo "round $round done"
done
