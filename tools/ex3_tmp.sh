set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ex7
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "kept_patch or every_launch_shape or full_size or larger_than or hint or seeded" > gpurun_out/ex7/tests.log 2>&1 || { tail -30 gpurun_out/ex7/tests.log; exit 1; }
tail -2 gpurun_out/ex7/tests.log
for R in 1 2; do
timeout -k 10 300 python tools/tune.py --workload 1500 --rounds 5 --bpc 8 --variants "16,2,2,0,18,1,24:16,2,2,6,18,1,24" | cut -c1-100 || exit 1
timeout -k 10 300 python tools/tune.py --workload imix --rotate 3 --rounds 5 --bpc 8 --variants "16,2,2,0,18,1,24:16,2,2,6,18,1,24" | cut -c1-100 || exit 1
done
