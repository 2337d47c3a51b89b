set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03j
timeout -k 10 600 python -u -m pytest tests/test_gpu_pq.py tests/test_gpu_param_capacity.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03j/tests.log 2>&1
SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so timeout -k 10 300 python3 -u tools/pqprobe.py 8000000 0 > gpurun_out/r03j/pq_v0.log 2>&1
timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03j/cfg.json 50,3 > gpurun_out/r03j/cfg.log 2>&1
SG_DEBUG_FLAGS=128 timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03j/cfg16.json 50 > gpurun_out/r03j/cfg16.log 2>&1
SG_VARIANT=1 SG_PROF_BIN=0 SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so timeout -k 10 300 python3 -u tools/hotprobe.py 3 8000000 2 > gpurun_out/r03j/c3_bin0.log 2>&1
echo ok
