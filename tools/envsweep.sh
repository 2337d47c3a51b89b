#!/bin/bash
# bench.py under several engine env settings: one JSON line per setting in gpurun_out/$TAG/
# usage: tools/envsweep.sh TAG "ENV=1 ENV2=2" "ENV=..." ...
set -e
TAG=${1:-envsweep}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for SET in "$@"; do
  i=$((i+1))
  env $SET timeout -k 10 240 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $OUT/run$i.json 2> $OUT/run$i.err
  echo "$SET" > $OUT/run$i.env
done
echo sweep done
