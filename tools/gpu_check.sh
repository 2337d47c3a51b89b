#!/bin/bash
# One GPU call: parity tests, bench, rocprof kernel-trace summary.  Every GPU step has its own
# time limit and the steps are chained so the first failure ends the call.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
echo done
