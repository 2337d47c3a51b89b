set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03t/tests.log 2>&1
bash tools/variants.sh r03t_ab base d8f > gpurun_out/r03t_ab.txt 2>&1
cat gpurun_out/r03t_ab.txt
timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03t/cfg.json 2,3,50 > gpurun_out/r03t/cfg.log 2>&1
python3 -c "
import json,sys
for c in json.load(open(sys.argv[1]))['configs']: print(c['config'][:3], round(c['value']/1e6,1), 'M/s', round(c['ms_per_batch'],2))" gpurun_out/r03t/cfg.json
