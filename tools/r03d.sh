set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/bench_prof.sh r03d $1
bash tools/timeline.sh r03d_tl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03d_c3 -o run -- python3 tools/config_bench.py gpurun_out/r03d_c3.json 3 > gpurun_out/r03d_c3.log 2>&1
echo ok
