set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b_pytest.log 2>&1
SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so SG_DEBUG=1 timeout -k 10 300 python -u tools/hotprobe.py 4 16400000 2 > gpurun_out/r02b_hotprobe.log 2>&1
echo done
