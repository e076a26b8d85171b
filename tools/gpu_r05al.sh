# round-5: strong-scaling projection of the final f64 headline (each rank's share timed on one GPU)
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python tools/rank_split_time.py --precision f64 --ns 1,2,4,8 --reps 3 > $OUT/rank_split_r05al.jsonl 2> $OUT/rank_split_r05al.err || exit $?
