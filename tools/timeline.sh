#!/bin/bash
# Kernel timelines of bench.py (rocprofv3 --kernel-trace, full CSV) with and without the two-stage
# pipeline, for tools/timeline.py.  usage: tools/timeline.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-tl}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --sub-batches 2 --no-cpu-baseline --no-configs"
SG_PIPELINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/serial -o run -- python3 bench.py $ARGS > $OUT/serial.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/pipe -o run -- python3 bench.py $ARGS > $OUT/pipe.log 2>&1
echo timeline done
