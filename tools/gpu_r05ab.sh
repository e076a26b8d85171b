# round-5: lane / pass counts of the f64 walk's owner phase (RTW_PROF build)
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python tools/lane_profile.py run --config C5 --precision f64 --spp 16 >> $OUT/lanes_r05ab.jsonl 2>> $OUT/lanes_r05ab.err || exit $?
timeout -k 10 200 python tools/lane_profile.py run --config C3 --precision f64 --spp 64 >> $OUT/lanes_r05ab.jsonl 2>> $OUT/lanes_r05ab.err || exit $?
