set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests/test_gpu_pq.py tests/test_gpu_param_capacity.py tests/test_gpu_parity.py -k "pq or param or c5 or exit_with_args" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03m/tests.log 2>&1
SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so timeout -k 10 300 python3 -u tools/pqprobe.py 8000000 0 > gpurun_out/r03m/pq_v0.log 2>&1
timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03m/cfg.json 50,5 > gpurun_out/r03m/cfg.log 2>&1 || true
echo ok
