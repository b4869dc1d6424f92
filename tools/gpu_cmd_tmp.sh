set -o pipefail
for r in 1 2 3; do
  for L in xsknf_amd/lib build/nohalf; do
    XSKNF_GPU_LIB=$PWD/$L/libxsknf_gpu.so timeout -k 10 200 python tools/tune.py --workload imix --rotate 4 --bpc 4 --rounds 4 --variants 16,2,2,0,18,1,56 2>>gpurun_out/imix_nh.err | sed "s|^{|{\"lib\": \"$L\", |" >> gpurun_out/imix_nh.jsonl || exit 1
  done
done
cut -c1-200 gpurun_out/imix_nh.jsonl
