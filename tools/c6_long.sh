#!/bin/bash
# C6 over more batches (pool growth and compactions in the timed region)
set -e
timeout -k 10 400 python tools/extprof.py c6 ${1:-6} > gpurun_out/c6long.log 2>&1
