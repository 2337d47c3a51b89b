set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03v
for cfg in "SG_X=0" "SG_PQ_WIDE=1000000000" "SG_DEBUG_FLAGS=128" "SG_PQ_WIDE=32768"; do
  n=$(echo "$cfg" | tr ' =' '__')
  env $cfg timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03v/c5_$n.json 50 > gpurun_out/r03v/c5_$n.log 2>&1
  python3 -c "
import json,sys
for c in json.load(open(sys.argv[1]))['configs']: print(sys.argv[2], c['config'][:3], round(c['value']/1e6,1), 'M/s', round(c['ms_per_batch'],2))" gpurun_out/r03v/c5_$n.json "$cfg"
done
bash tools/shard_rehearsal.sh r03v_sh 8 > gpurun_out/r03v/sh8.log 2>&1
cat gpurun_out/r03v/sh8.log
