set -e
export TMPDIR=/tmp
bash tools/shard_rehearsal.sh r03l 8 > gpurun_out/r03l_8.log 2>&1
cat gpurun_out/r03l_8.log
bash tools/shard_rehearsal.sh r03l 4 > gpurun_out/r03l_4.log 2>&1
cat gpurun_out/r03l_4.log
