set -e
bash tools/r03h.sh
bash tools/r03i.sh
