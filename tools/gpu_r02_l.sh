#!/bin/bash
# r02 step L: GPU tests, the default bench (with the f64 / plain-f32 mode lines
# and the CPU baseline), rank-split timing, then rocprofv3 kernel trace + PMC
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_v3}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/${T}_pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/${T}_pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 400 python -u bench.py > $OUT/${T}_bench.json 2> $OUT/${T}_bench.err || { tail -20 $OUT/${T}_bench.err; exit 1; }
cat $OUT/${T}_bench.json
timeout -k 10 300 python -u tools/rank_split_time.py --ns 1,2,4,8 --reps 3 > $OUT/${T}_rank_split.jsonl 2>&1 || { tail -5 $OUT/${T}_rank_split.jsonl; exit 1; }
grep nranks $OUT/${T}_rank_split.jsonl | cut -c1-200
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU;SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
  bash tools/profile.sh $T --steps 2 --warmup 1 --no-cpu-baseline --no-modes || exit $?
cd "$ROOT"
python3 tools/pmc_summary.py $OUT/prof_$T --traffic $OUT/${T}_traffic.json book1_simple_1200x800_500spp_depth50 > $OUT/${T}_pmc_summary.txt
cat $OUT/${T}_pmc_summary.txt
find $OUT/prof_$T -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/${T}_kernel_stats.csv
head -4 $OUT/${T}_kernel_stats.csv
