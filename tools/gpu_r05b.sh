set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_multidevice.py -v --timeout 120 --timeout-method thread > $OUT/pytest_md_r05b.log 2>&1; rc=$?
echo "md rc=$rc"; tail -3 $OUT/pytest_md_r05b.log
case $rc in 0|1) ;; *) exit $rc;; esac
for cfg in "C3 f64 0" "C5 f32 0" "C5 f64 64" "C2 f64 100"; do
  set -- $cfg
  timeout -k 10 200 python tools/clock_profile.py run --config $1 --precision $2 --spp $3 >> $OUT/clock_r05b.jsonl 2>> $OUT/clock_r05b.err || exit $?
  echo "clock $1 $2 done"
done
