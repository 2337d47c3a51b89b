set -e
export TMPDIR=/tmp
bash tools/quickbench.sh r03aa "SG_X=0" "SG_J1_MAX=2048" "SG_J1_MAX=1024" "SG_X=1" "SG_J1_MAX=2048"
