set -e
export TMPDIR=/tmp
bash tools/variants.sh r03q_ab base openj4 d8f r02 j1w2 > gpurun_out/r03q_ab.txt 2>&1
cat gpurun_out/r03q_ab.txt
