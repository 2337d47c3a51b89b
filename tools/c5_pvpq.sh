#!/bin/bash
# C5 with its one-rule heads through the value-parallel passes (SG_PV_PQ=1, default) and through k_pq (0)
set -e
out=${1:-gpurun_out/c5pvpq.log}
: > "$out"
for v in 1 0; do echo "== SG_PV_PQ=$v" >> "$out"; SG_PV_PQ=$v timeout -k 10 200 python tools/extprof.py c5 >> "$out" 2>&1; done
