set -o pipefail
cd $GRAFT_REPO_ROOT
BPC=8 bash tools/explore_step.sh ex4 imix "16,2,2,0,1,1,24:16,2,2,0,9,1,24:16,3,1,0,9,1,24:16,2,2,0,1,1,20:16,2,2,0,9,1,20" | cut -c1-120 || exit 1
timeout -k 10 400 env XSKNF_GPU_LIB=$GRAFT_REPO_ROOT/build/ab/libxsknf_gpu.so python tools/tune.py --workload imix --frames 8388608 --variants "16,2,2,0,9,1,24" --bpc 8 --rounds 3 | cut -c1-120 || exit 1
timeout -k 10 400 env XSKNF_GPU_LIB=$GRAFT_REPO_ROOT/build/ab/libxsknf_gpu.so python tools/tune.py --workload imix --frames 4194304 --variants "16,2,2,0,9,1,24" --bpc 8 --rounds 3 | cut -c1-120 || exit 1
