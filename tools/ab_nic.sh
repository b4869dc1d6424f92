set -o pipefail
export XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so
mkdir -p gpurun_out/ab
for ch in nic zero; do
timeout -k 10 200 python tools/tune.py --workload 64 --checks $ch --rotate 13 --rounds 7 --variants "1,4,1,0,1,0,128:1,4,1,0,1,0,160:1,5,2,0,1,0,32:1,4,1,0,1:1,4,2,0,1:1,5,1,0,1:1,4,1,0,1,0,2112:16,2,2,0,1,1,20:16,2,2,0,18,1,56" >> gpurun_out/ab/ab64_nic.txt || exit 1
done
timeout -k 10 200 python tools/tune.py --workload imix --checks nic --rotate 3 --rounds 7 --variants "16,2,2,0,18,1,56:16,2,2,0,18,1,20:16,2,2,0,1,1,24:16,3,1,0,1,1,24" >> gpurun_out/ab/ab64_nic.txt || exit 1
timeout -k 10 200 python tools/tune.py --workload 1500 --checks nic --rounds 5 --variants "16,2,2,0,18,1,24:16,2,2,0,1,1,56:16,3,2,0,18,1,24" >> gpurun_out/ab/ab64_nic.txt || exit 1
cat gpurun_out/ab/ab64_nic.txt
