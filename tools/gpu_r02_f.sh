#!/bin/bash
# r02 step F: new GPU tests (C4, PPM), C3/C5 timings, C5 PMC (HBM/MALL point)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_ppm.py -v -rA -s --timeout 300 --timeout-method thread > $OUT/pytest_c4_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|C4 rank" $OUT/pytest_c4_$T.log | tail -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/bench_configs.py --configs C3,C5 > $OUT/configs_$T.jsonl 2> $OUT/configs_$T.err
rc=$?; echo "configs rc=$rc"; cat $OUT/configs_$T.jsonl; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  ( cd /tmp && timeout -k 10 240 rocprofv3 --pmc $set -d "$ROOT/$OUT/prof_c5_$T/pmc$i" -o pmc --output-format csv \
      -- python3 "$ROOT/tools/bench_configs.py" --configs C5 --spp-scale 0.25 > "$ROOT/$OUT/prof_c5_${T}_pmc$i.log" 2>&1 )
  rc=$?; echo "c5 pmc$i ($set) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_c5_$T" -o trace --output-format csv \
    -- python3 "$ROOT/tools/bench_configs.py" --configs C5 --spp-scale 0.25 > "$ROOT/$OUT/prof_c5_${T}_trace.log" 2>&1 )
echo "c5 trace rc=$?"
python3 tools/pmc_summary.py $OUT/prof_c5_$T --traffic $OUT/${T}_c5_traffic.json c5_1M_spheres_1920x1080_64spp_depth50 > $OUT/${T}_c5_pmc_summary.txt
cat $OUT/${T}_c5_pmc_summary.txt $OUT/${T}_c5_traffic.json; cat $OUT/prof_c5_$T/trace_kernel_stats.csv | cut -c1-150
