set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w/tests.log 2>&1
bash tools/bench_prof.sh r03w $1
bash tools/shard_rehearsal.sh r03w_sh 8 > gpurun_out/r03w/sh8.log 2>&1
cat gpurun_out/r03w/sh8.log
