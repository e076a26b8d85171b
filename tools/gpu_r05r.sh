# round-5: lane occupancy of the f32 cooperative walk (RTW_PROF build)
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python tools/lane_profile.py run --config C5 --spp 32 >> $OUT/lanes_r05r.jsonl 2>> $OUT/lanes_r05r.err || exit $?
timeout -k 10 200 python tools/lane_profile.py run --config C3 --spp 64 >> $OUT/lanes_r05r.jsonl 2>> $OUT/lanes_r05r.err || exit $?
