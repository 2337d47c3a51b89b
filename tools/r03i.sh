set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03i
for b in 0 1 2; do
SG_VARIANT=1 SG_PROF_BIN=$b SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so timeout -k 10 300 python3 -u tools/hotprobe.py 3 8000000 2 > gpurun_out/r03i/c3_bin$b.log 2>&1
done
echo ok
