#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (MI355X_MICROARCH.md: they cannot share a pass).  Every GPU step has its own limit.
# usage: tools/profile.sh TAG [GIT_HEAD]   -> gpurun_out/TAG/{kernel_stats.csv,pmc.json}
set -e
export TMPDIR=/tmp
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --sub-batches 2 --no-cpu-baseline --no-configs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
STATS=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
cp $STATS $OUT/kernel_stats.csv
python3 tools/pmc_summary.py $(find $OUT/fetch -name '*counter_collection.csv' | head -1) \
    $(find $OUT/write -name '*counter_collection.csv' | head -1) $OUT/kernel_stats.csv $OUT/pmc.json ${2:-}
echo profile done
