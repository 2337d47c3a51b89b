set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u/tests.log 2>&1
bash tools/bench_prof.sh r03u $1
bash tools/variants.sh r03u_ab base d8f > gpurun_out/r03u_ab.txt 2>&1
cat gpurun_out/r03u_ab.txt
