# round-5: hit64 f64 Lambertian direction with the azimuth's sin / cos in f32 (trig32) -- timing and the f32 tolerance
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python tools/ab_bench.py --variants tree,trig32 --modes f32 --rounds 2 > $OUT/ab_trig32_r05ak.jsonl 2> $OUT/ab_trig32_r05ak.err || exit $?
RTW_LIB_OVERRIDE=build/variants/trig32/librtw.so timeout -k 10 300 python tools/f32_tolerance.py >> $OUT/tol_trig32_r05ak.jsonl 2>> $OUT/tol_trig32_r05ak.err || exit $?
