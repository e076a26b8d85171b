set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3_c5.py tests/test_gpu_multidevice.py -v --timeout 200 --timeout-method thread > $OUT/pytest_r05h.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_r05h.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_ab_walk.sh old remerge cmax12 ntnode || exit $?
bash tools/gpu_r05g.sh
