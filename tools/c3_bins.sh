#!/bin/bash
# C3 under several J4 bin limits (tools/extprof.py c3), one line per setting in gpurun_out/$TAG/
set -e
TAG=${1:-c3bins}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for J4 in 65536 16384 4096; do
  SG_J4_MAX=$J4 timeout -k 10 200 python3 tools/extprof.py c3 > $OUT/j4_$J4.log 2>&1
  tail -1 $OUT/j4_$J4.log
done
echo sweep done
