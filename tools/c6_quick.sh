#!/bin/bash
# C6 at the default settings (tools/extprof.py c6) and a kernel-trace profile of it
set -e
out=${1:-gpurun_out/c6quick.log}
timeout -k 10 200 python tools/extprof.py c6 3 > "$out" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pvprof -o pv -- python tools/extprof.py c6 2 > gpurun_out/pvprof.log 2>&1
