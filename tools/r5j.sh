# round 5: SLP A/B + attention repro under load + race traces (one call), then proxies in r5k.sh
set -e
bash tools/r5i.sh
bash tools/r5h.sh
