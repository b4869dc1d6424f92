set -o pipefail
cd $GRAFT_REPO_ROOT
export XSKNF_GPU_LIB=$GRAFT_REPO_ROOT/build/ab/libxsknf_gpu.so
timeout -k 10 400 python tools/tune.py --workload imix --rotate 3 --rounds 5 --bpc 4,8 --variants "16,2,2,0,18,1,24:16,3,1,0,18,1,24:16,2,2,0,18,1,20:16,3,2,0,18,1,20:16,2,1,0,18,1,24" | cut -c1-112 || exit 1
timeout -k 10 400 python tools/tune.py --workload 64 --rotate 13 --rounds 5 --bpc 8 --variants "16,2,2,0,18,1,20:1,5,2,0,1:1,6,2,0,1:1,5,2,0,5:1,7,2,0,1:16,2,2,0,17,1,20" | cut -c1-112 || exit 1
