set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
for t in "lpt_pilot_spp=2" "lpt_pilot_spp=1" "lpt_pilot_spp=2,lpt_pilot_depth=12" "lpt_pilot_spp=1,lpt_pilot_depth=12" "lpt_pilot_spp=1,lpt_pilot_depth=6"; do
  timeout -k 10 200 python -u tools/rank_split_time.py --ns 1,8 --reps 3 --tuning $t 2>&1 | grep size | cut -c1-330 || exit 1
done
for v in tree nosteal; do
  echo "== $v C3,C5 full"
  if [ "$v" = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so; fi
  timeout -k 10 300 python -u tools/bench_configs.py --configs C3,C5 2>&1 | cut -c1-300 | grep config || exit 1
done
