#!/bin/bash
# Bin-threshold sweep: bench line + rocprofv3 kernel stats per SG_LANE_MAX / SG_J1_MAX setting.
set -e
export TMPDIR=/tmp
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for LM in ${LANES:-256 64 32}; do
  SG_LANE_MAX=$LM timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lm$LM -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/lm$LM.json 2> $OUT/lm$LM.err
done
echo sweep done
