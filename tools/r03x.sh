set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03x
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x/tests.log 2>&1
bash tools/bench_prof.sh r03x $1
