#!/bin/bash
# Kernel durations of one rank's shard (bench.py --shard R/N, alone on one GPU) and the phase counters of
# its J16 and J4 owners (SG_DEBUG=1, SG_PROF_BIN).  usage: tools/shard_profile.sh TAG R N
set -e
export TMPDIR=/tmp
TAG=$1; R=$2; N=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 bench.py --shard $R/$N --steps 2 --warmup 1 --no-cpu-baseline --max-sub-batches 4 --base-batches 4 > $OUT/tr.log 2>&1
cp $(find $OUT/tr -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
python3 tools/timeline.py $(find $OUT/tr -name '*kernel_trace.csv' | head -1) --window > $OUT/timeline.txt
rm -rf $OUT/tr
head -14 $OUT/kernel_stats.csv | cut -d, -f1-4
echo shard profile done
