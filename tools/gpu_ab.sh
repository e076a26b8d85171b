#!/bin/bash
# GPU tests with the in-tree library, then tools/ab_bench.py over variants
# (build/variants/<name>, "tree" = in-tree) and CONFIGS (C3,C5) per variant.
#   tools/gpu_ab.sh TAG "v1,tree" ["f32,plain,f64"]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
T=$1; V=$2; M=${3:-f32,plain,f64}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${T}_pytest.log 2>&1
  rc=$?; tail -2 $OUT/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/${T}_pytest.log | head -30; exit $rc; }
fi
timeout -k 10 900 python -u tools/ab_bench.py --variants "$V" --modes "$M" --rounds ${ROUNDS:-2} > $OUT/${T}_ab.jsonl 2>&1
rc=$?; cat $OUT/${T}_ab.jsonl; [ $rc -eq 0 ] || exit $rc
if [ -n "${CONFIGS:-}" ]; then for v in ${V//,/ }; do
  echo "== $v $CONFIGS"
  if [ "$v" = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so; fi
  timeout -k 10 300 python -u tools/bench_configs.py --configs $CONFIGS --spp-scale ${SPP_SCALE:-0.25} 2>&1 | cut -c1-330 | grep config || exit 1
done; fi
