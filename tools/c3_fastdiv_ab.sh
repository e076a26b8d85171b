cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do for v in tree nofd64; do
  if [ "$v" = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so; fi
  echo "== $r $v"
  timeout -k 10 300 python -u tools/bench_configs.py --configs C3 --precision f64 --spp-scale 0.5 --steps 2 2>&1 | grep -o '"kernel_ms[^,]*,' || exit 1
done; done
