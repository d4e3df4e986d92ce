set -e
bash tools/r5d.sh
bash tools/r5e.sh
