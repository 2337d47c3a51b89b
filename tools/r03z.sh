set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03z
for v in base tg1 tg3 base; do
  if [ $v = base ]; then L=""; else L=$PWD/var/lib_$v.so; fi
  SG_LIB_PATH=$L timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03z/cfg_$v.json 3 > gpurun_out/r03z/cfg_$v.log 2>&1
  python3 -c "
import json,sys
for c in json.load(open(sys.argv[1]))['configs']: print(sys.argv[2], c['config'][:3], round(c['value']/1e6,1), 'M/s', round(c['ms_per_batch'],2))" gpurun_out/r03z/cfg_$v.json $v
done
