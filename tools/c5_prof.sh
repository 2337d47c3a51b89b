#!/bin/bash
# C5 kernel-trace profile (tools/extprof.py c5)
set -e
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o c5 -- python tools/extprof.py c5 > gpurun_out/c5prof.log 2>&1
