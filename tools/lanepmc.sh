#!/bin/bash
# SQ / cache counters of the decide kernels (one --pmc pass each, own time limit).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-lanepmc}
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $OUT/cache -o run -- python3 bench.py $ARGS > $OUT/cache.log 2>&1
echo pmc done
