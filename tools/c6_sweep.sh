#!/bin/bash
# C6 decide-stage knobs, one extprof run each (tools/extprof.py c6): the value-parallel passes and the lane bound;
# then a kernel-trace profile of the default
set -e
out=${1:-gpurun_out/c6sweep.log}
: > "$out"
run() { echo "== $*" >> "$out"; env "$@" timeout -k 10 200 python tools/extprof.py c6 3 >> "$out" 2>&1; }
run SG_PV=1
run SG_PV=1 SG_LANE_MAX=64
run SG_PV=1 SG_LANE_MAX=128
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pvprof -o pv -- python tools/extprof.py c6 2 > gpurun_out/pvprof.log 2>&1
