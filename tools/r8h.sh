# round 5 final tree: whole GPU suite + smoke
mkdir -p gpurun_out
TAG=r8h bash tools/gpu.sh tests smoke || exit 1
