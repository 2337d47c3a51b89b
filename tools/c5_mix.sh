#!/bin/bash
# C5 with its param-only programs as k_pq's (default) and as XF_MIX (SG_MIX_PQ=1: value-parallel passes + owners)
set -e
out=${1:-gpurun_out/c5mix.log}
: > "$out"
for v in 0 1; do echo "== SG_MIX_PQ=$v" >> "$out"; SG_MIX_PQ=$v timeout -k 10 200 python tools/extprof.py c5 >> "$out" 2>&1; done
