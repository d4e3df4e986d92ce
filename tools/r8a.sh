# round 5 re-entry validation of HEAD (freshly rebuilt extensions): whole GPU suite + smoke
mkdir -p gpurun_out
TAG=r8a bash tools/gpu.sh tests smoke || exit 1
