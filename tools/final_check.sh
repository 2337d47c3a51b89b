#!/bin/bash
# round-end evidence in one call: the GPU suite, smoke, rocprof kernel stats + HBM PMC, the bench line
set -e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests_fc.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_fc.log 2>&1
timeout -k 10 700 tools/profile.sh ${1:-r04l} > gpurun_out/prof_fc.log 2>&1
timeout -k 10 480 python bench.py > gpurun_out/bench_fc.json 2> gpurun_out/bench_fc.log
