set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03k/tests.log 2>&1
timeout -k 10 300 python3 -u tools/config_bench.py gpurun_out/r03k/cfg.json 3,50 > gpurun_out/r03k/cfg.log 2>&1
bash tools/quickbench.sh r03k/ab "SG_X=0" "SG_DEBUG_FLAGS=64"
SG_VARIANT=1 SG_PROF_BIN=0 SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so timeout -k 10 300 python3 -u tools/hotprobe.py 3 8000000 2 > gpurun_out/r03k/c3_bin0.log 2>&1
echo ok
