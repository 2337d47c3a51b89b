#!/bin/bash
# per-config rocprofv3 passes (kernel stats, FETCH_SIZE, WRITE_SIZE) -> profiles/pmc_configs.json (copied to gpurun_out)
set -e
export TMPDIR=/tmp
GH=$1; shift
for C in "$@"; do
  O=gpurun_out/cfg_$C; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --only-config $C > $O/trace.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --only-config $C > $O/fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --only-config $C > $O/write.log 2>&1
  cp $(find $O/trace -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
  python3 tools/pmc_configs.py $C $(find $O/fetch -name '*counter_collection.csv' | head -1) $(find $O/write -name '*counter_collection.csv' | head -1) $O/kernel_stats.csv $GH
  cp profiles/pmc_configs.json gpurun_out/pmc_configs.json
  echo "$C done"
done
