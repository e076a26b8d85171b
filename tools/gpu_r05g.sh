set -u
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_piece_sweep.sh || exit $?
for v in tree lamb64; do
  if [ $v = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=build/variants/$v/librtw.so; fi
  timeout -k 10 300 python tools/f32_tolerance.py >> $OUT/f32tol_r05g.jsonl 2>> $OUT/f32tol_r05g.err || exit $?
  timeout -k 10 200 python tools/sweep.py --precision f32 --grid "hit64=1" --rounds 3 >> $OUT/sweep_r05g_$v.log 2>&1 || exit $?
  echo "$v done"
done

