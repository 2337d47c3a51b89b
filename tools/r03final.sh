set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03final
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03final/smoke.log 2>&1
/usr/bin/time -v timeout -k 10 900 python -u bench.py > gpurun_out/r03final/bench.json 2> gpurun_out/r03final/bench.err
tail -1 gpurun_out/r03final/smoke.log
python3 -c "import json;d=json.load(open('gpurun_out/r03final/bench.json'));print(d['value']/1e9, d['steps'], d['warmup'], d['ms_per_step'], d['roofline']['traffic'], [round(c['value']/1e6,1) for c in d['configs']])"
grep "Elapsed" gpurun_out/r03final/bench.err
