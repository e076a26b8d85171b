set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 200 --timeout-method thread > $OUT/pytest_gpu_r05i.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu_r05i.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_ab_walk.sh old remerge kargs || exit $?
