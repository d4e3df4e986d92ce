# round 5: board power / clock over the headline step (tools/step_power.py)
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/step_power.py --steps 8 --warmup 3 > gpurun_out/step_power_r8f.log 2>&1 || exit 1
