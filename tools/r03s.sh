set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s
bash tools/variants.sh r03s_ab j16w8 j1w3 d8f openj4 > gpurun_out/r03s_ab.txt 2>&1
cat gpurun_out/r03s_ab.txt
for v in j16w8 j1w3; do
  SG_LIB_PATH=$PWD/var/lib_$v.so timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03s/cfg_$v.json 2,3 > gpurun_out/r03s/cfg_$v.log 2>&1
  python3 -c "
import json,sys
for c in json.load(open(sys.argv[1]))['configs']: print(sys.argv[2], c['config'][:3], round(c['value']/1e6,1), 'M/s', round(c['ms_per_batch'],2))" gpurun_out/r03s/cfg_$v.json $v
done
