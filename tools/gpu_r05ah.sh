# round-5: LLVM scheduling strategies (max-ilp, max-memory-clause) on the C2 kernels
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python tools/ab_bench.py --variants tree,milp,mmc --modes f64,f32 --rounds 2 > $OUT/ab_sched_r05ah.jsonl 2> $OUT/ab_sched_r05ah.err || exit $?
