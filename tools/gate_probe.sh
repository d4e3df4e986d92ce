#!/bin/bash
# both gate kinds; stops at a time limit / signal exit (>= 124), a clean failure (1) goes on to the next kind
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for k in 1 0; do
    timeout -k 5 30 python -u tools/gate_probe.py $k >> gpurun_out/gate_probe.log 2>&1
    rc=$?
    echo "kind $k rc $rc" >> gpurun_out/gate_probe.log
    [ $rc -ge 124 ] && exit $rc
done
exit 0
