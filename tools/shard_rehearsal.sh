#!/bin/bash
# Per-rank step time of an N-GPU strong-scaling bench, rehearsed on one GPU: every rank's shard of the
# C4 trace (bench.py --shard R/N) run alone, one after another.  The N-GPU step is the slowest rank's
# (plus the MetricNode all-gather); this is a prediction, never a measurement of the N-GPU run.
# usage: [SHARDING=hash] [RANKB=global] [ALPHA=0.9] tools/shard_rehearsal.sh TAG N [N ...]   (default: the balanced resource table)
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for N in "$@"; do
    for R in $(seq 0 $((N - 1))); do
        timeout -k 10 200 python bench.py --shard $R/$N --steps 3 --warmup 1 --no-cpu-baseline --no-configs --sub-batches 16 --base-batches 8 ${SHARDING:+--sharding $SHARDING} ${RANKB:+--rank-batches $RANKB} ${ALPHA:+--balance-alpha $ALPHA} > $OUT/s${R}_of_$N.json 2> $OUT/s${R}_of_$N.err
    done
    python3 - $OUT $N <<'PY'
import json, sys
out, n = sys.argv[1], int(sys.argv[2])
rows = [json.load(open("%s/s%d_of_%d.json" % (out, r, n))) for r in range(n)]
ms = [d["roofline"]["batch_ms"] for d in rows]
ent = sum(d["value"] * d["roofline"]["batch_ms"] / 1e3 for d in rows)  # entries per global batch, all ranks
print("N=%d per-rank ms per global batch: %s  -> slowest %.3f ms, predicted node rate %.2f G entries/s"
      % (n, " ".join("%.3f" % x for x in ms), max(ms), ent / (max(ms) / 1e3) / 1e9))
PY
done
echo rehearsal done
