set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03final
t0=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r03final/bench.json 2> gpurun_out/r03final/bench.err
t1=$(date +%s)
python3 -c "import json;d=json.load(open('gpurun_out/r03final/bench.json'));print(d['value']/1e9, d['steps'], d['warmup'], d['ms_per_step'], d['roofline']['traffic'], [round(c['value']/1e6,1) for c in d['configs']])"
echo "bench wall $((t1 - t0)) s"
