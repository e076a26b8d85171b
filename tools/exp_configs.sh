set -u
cd "$GRAFT_REPO_ROOT"
for v in base exp1 exp2 exp4; do
  echo "== $v"
  RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so timeout -k 10 300 python tools/bench_configs.py --configs C5,C3 --spp-scale 0.5 --steps 2 || exit $?
done
