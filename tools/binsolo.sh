#!/bin/bash
# Kernel timeline with every decide kernel alone on the GPU (SG_PIPELINE=0, SG_DEBUG_FLAGS=8).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-solo}
mkdir -p $OUT
SG_PIPELINE=0 SG_DEBUG_FLAGS=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/solo -o run -- python3 bench.py --steps 2 --warmup 1 --sub-batches 2 --no-cpu-baseline > $OUT/solo.log 2>&1
echo solo done
