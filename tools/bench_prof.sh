#!/bin/bash
# One GPU call: smoke, the driver's bench line (C4 + C2/C3/C5 sub-lines), then the rocprof passes.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
bash tools/profile.sh ${TAG}_prof ${2:-}
echo done
