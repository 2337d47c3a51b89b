#!/bin/bash
# Short bench lines (no CPU baseline) for a list of environment settings, one JSON per setting, plus
# a one-line summary each: G entries/s, ms per batch, group / decide ms.  usage: tools/quickbench.sh TAG "ENV..." ...
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for cfg in "$@"; do
    n=$(echo "$cfg" | tr ' =' '__')
    env $cfg timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs > $OUT/$n.json 2> $OUT/$n.err
    python -c "import json,sys;d=json.load(open(sys.argv[1]));p=d['pipeline'];print(sys.argv[2], round(d['value']/1e9,3),round(p['wall_ms_per_batch'],3),round(p['group_ms'],3),round(p['decide_ms'],3))" $OUT/$n.json "$cfg"
done
