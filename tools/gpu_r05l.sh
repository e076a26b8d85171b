# round-5 diagnostic A/B of the f64 headline's specular pass (variants built in build/variants)
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python tools/ab_bench.py --variants tree,nomloop,nomat,rcpdiv --modes f64 --rounds 2 \
  > $OUT/ab_spec_r05l.jsonl 2> $OUT/ab_spec_r05l.err || exit $?
