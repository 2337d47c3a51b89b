# C5 diagnosis: kernel stats of the bench's C5 sub-line shape, k_pq vs the per-lane path, PQ16 threshold
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03e/pq -o run -- python3 tools/config_bench.py gpurun_out/r03e/pq.json 50 > gpurun_out/r03e/pq.log 2>&1
SG_PQ_WIDE=1000000000 timeout -k 10 300 python3 tools/config_bench.py gpurun_out/r03e/pq_narrow.json 50 > gpurun_out/r03e/pq_narrow.log 2>&1
SG_PQ=0 timeout -k 10 300 python3 tools/config_bench.py gpurun_out/r03e/lane.json 50 > gpurun_out/r03e/lane.log 2>&1
echo ok
