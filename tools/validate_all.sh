#!/bin/bash
# parity of the param paths, C6 timing + profile, then the rocprof evidence and the bench line (one call)
set -e
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pq.py tests/test_gpu_mix.py tests/test_gpu_param_capacity.py tests/test_gpu_parity.py > gpurun_out/va_tests.log 2>&1
timeout -k 10 450 tools/c6_quick.sh gpurun_out/c6quick.log
timeout -k 10 700 tools/profile.sh ${1:-r04k} > gpurun_out/prof_va.log 2>&1
timeout -k 10 480 python bench.py > gpurun_out/bench_va.json 2> gpurun_out/bench_va.log
