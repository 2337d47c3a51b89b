set -e
export TMPDIR=/tmp
bash tools/quickbench.sh r03p "SG_X=0" "SG_J1_MAX=2048" "SG_J1_MAX=1024" "SG_J4_MAX=32768" "SG_LANE_MAX=128"
bash tools/variants.sh r03p_ab j1w2 > gpurun_out/r03p_ab.txt 2>&1
cat gpurun_out/r03p_ab.txt
