set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03r
bash tools/variants.sh r03r_ab base openj4 noopen c7e d8f > gpurun_out/r03r_ab.txt 2>&1
cat gpurun_out/r03r_ab.txt
for v in base openj4 d8f; do
  if [ $v = base ]; then L=""; else L=$PWD/var/lib_$v.so; fi
  SG_LIB_PATH=$L timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03r/cfg_$v.json 2,3 > gpurun_out/r03r/cfg_$v.log 2>&1
  python3 -c "
import json,sys
for c in json.load(open(sys.argv[1]))['configs']: print(sys.argv[2], c['config'][:3], round(c['value']/1e6,1), 'M/s', round(c['ms_per_batch'],2))" gpurun_out/r03r/cfg_$v.json $v
done
