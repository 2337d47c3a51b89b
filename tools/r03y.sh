set -e
export TMPDIR=/tmp
bash tools/variants.sh r03y_ab base j1s base j1s > gpurun_out/r03y_ab.txt 2>&1
cat gpurun_out/r03y_ab.txt
