set -o pipefail
bash tools/prof_all.sh r06 1500 imix 64 jumbo config4 1500-nic imix-nic 64-nic jumbo-nic 64-13M && du -sh gpurun_out
