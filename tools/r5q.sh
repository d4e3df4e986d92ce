bash tools/r5o.sh
bash tools/r5p.sh
