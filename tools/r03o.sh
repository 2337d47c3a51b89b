set -e
export TMPDIR=/tmp
bash tools/r03m.sh
bash tools/variants.sh r03o_ab base r02 > gpurun_out/r03o_ab.txt 2>&1
cat gpurun_out/r03o_ab.txt
bash tools/r03l.sh
