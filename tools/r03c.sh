set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_shape.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c_pytest.log 2>&1
bash tools/quickbench.sh r03c_ab "SG_X=0" "SG_DEBUG_FLAGS=64" "SG_X=1"
timeout -k 10 300 python -u tools/config_bench.py gpurun_out/r03c_cfg_open.json 2,3 > gpurun_out/r03c_cfg_open.log 2>&1
SG_DEBUG_FLAGS=64 timeout -k 10 300 python -u tools/config_bench.py gpurun_out/r03c_cfg_closed.json 2,3 > gpurun_out/r03c_cfg_closed.log 2>&1
echo ok
