#!/bin/bash
# One GPU call: parity tests, smoke, bench (driver config), rocprof kernel-trace + PMC passes.
# Every GPU step has its own time limit and the steps are chained so the first failure ends the call.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-run}
SEL=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $SEL > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
bash tools/profile.sh ${TAG}_prof ${3:-}
echo done
