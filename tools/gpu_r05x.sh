# round-5: the headline at chunk >= spp (every pixel's samples in one work item: no per-sample sums, no fold)
set -u
OUT=gpurun_out; mkdir -p $OUT
for t in "" "chunk=500" "" "chunk=500"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-modes --configs none ${t:+--tuning $t} >> $OUT/chunk_r05x.jsonl 2>> $OUT/chunk_r05x.err || exit $?
done
