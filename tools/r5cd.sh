set -e
bash tools/r5c.sh
bash tools/r5d.sh
