#!/bin/bash
# A/B of engine builds: for each library (base = the in-tree build, else var/lib_NAME.so) one short
# bench line and one rocprofv3 kernel-stats pass; prints G entries/s, ms per batch, group / decide ms
# and the average duration of the main kernels.  usage: tools/variants.sh TAG base NAME NAME@--batch-events,67108864 ...
# (after @: extra bench.py arguments and SG_* environment settings, commas for spaces)
set -e
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in "$@"; do
    name=${spec%%@*}
    XA=""; XE=""
    if [ "$spec" != "$name" ]; then
        for tok in $(echo "${spec#*@}" | tr ',' ' '); do
            case "$tok" in SG_*=*) XE="$XE $tok" ;; *) XA="$XA $tok" ;; esac
        done
    fi
    v=$(echo "$spec" | tr '@, ' '___')
    if [ "$name" = base ]; then LIB=""; else LIB="$PWD/var/lib_$name.so"; fi
    env $XE SG_LIB_PATH=$LIB timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs $XA > $OUT/$v.json 2> $OUT/$v.err
    env $XE SG_LIB_PATH=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$v -o run -- python3 bench.py --steps 2 --warmup 1 --sub-batches 2 --no-cpu-baseline --no-configs $XA > $OUT/tr_$v.log 2>&1
    cp $(find $OUT/tr_$v -name '*kernel_stats.csv' | head -1) $OUT/ks_$v.csv
    rm -rf $OUT/tr_$v
    python3 - "$OUT/$v.json" "$OUT/ks_$v.csv" "$v" <<'EOF'
import csv, json, sys
d = json.load(open(sys.argv[1])); p = d["pipeline"]
ks = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(sys.argv[2]))}
top = sorted(ks.items(), key=lambda x: -x[1])[:12]
print(sys.argv[3], "G/s %.3f batch %.3f group %.3f decide %.3f post %.3f" % (d["value"] / 1e9, p["wall_ms_per_batch"], p["group_ms"], p["decide_ms"], p["post_ms"]))
print("   ", ", ".join("%s %.0f" % (k.replace("void ", ""), v) for k, v in top))
EOF
done
echo variants done
