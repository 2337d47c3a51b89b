set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so timeout -k 10 300 python3 -u tools/pqprobe.py 8000000 0 > gpurun_out/r03f/pq_v0.log 2>&1
SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so timeout -k 10 300 python3 -u tools/pqprobe.py 8000000 14 > gpurun_out/r03f/pq_v14.log 2>&1
echo ok
