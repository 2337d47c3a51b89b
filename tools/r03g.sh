set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so timeout -k 10 300 python3 -u tools/pqprobe.py 8000000 0 > gpurun_out/r03g/pq_v0.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g/parity.log 2>&1
timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03g/c3.json 3 > gpurun_out/r03g/c3.log 2>&1
echo ok
