set -o pipefail
cd $GRAFT_REPO_ROOT
export XSKNF_GPU_LIB=$GRAFT_REPO_ROOT/build/ab_t2/libxsknf_gpu.so
timeout -k 10 500 python tools/tune.py --workload jumbo --rounds 5 --bpc 8 --reps 5 --variants "16,3,2,0,18,1,20:16,2,2,0,18,1,20:16,2,2,0,18,1,24:16,3,2,0,18,1,24:16,2,2,0,0,1,24" | cut -c1-110 || exit 1
