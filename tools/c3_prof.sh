#!/bin/bash
# C3 kernel-trace profile (tools/extprof.py c3, bench.py's C3 sub-line): stats plus the rocpd db for
# tools/rocpd_timeline.py.  usage: tools/c3_prof.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-c3prof}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o c3 -- python3 tools/extprof.py c3 > gpurun_out/$TAG/run.log 2>&1
echo c3 profile done
