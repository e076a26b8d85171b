#!/bin/bash
# GPU tests, then C3 / C5 timing in both precisions and the PMC passes of
# their kernels (tools/gpu_prof_c3.sh), each profile tagged TAG_C3_f64 etc.
#   tools/gpu_c3c5_round.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; TAG=$1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || exit $rc
for prec in f64 f32; do
  timeout -k 10 300 python -u tools/bench_configs.py --configs C3,C5 --precision $prec --steps 2 > "$OUT/${TAG}_configs_$prec.jsonl" 2>&1 || exit $?
  grep -o '"config": "[^"]*"\|"kernel_ms[^,]*' "$OUT/${TAG}_configs_$prec.jsonl"
done
if [ "${PROFILE:-1}" = 1 ]; then
  for cfg in C3 C5; do for prec in f64 f32; do
    bash tools/gpu_prof_c3.sh "${TAG}_${cfg}_${prec}" $cfg $prec > "$OUT/${TAG}_${cfg}_${prec}_prof.log" 2>&1 || exit $?
    echo "profiled $cfg $prec"
  done; done
fi
