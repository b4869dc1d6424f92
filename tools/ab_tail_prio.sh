set -o pipefail
mkdir -p gpurun_out/abtp
for r in 1 2; do
 for L in xsknf_amd/lib build/ab_t3 build/ab_p3; do
  for W in 1500 imix; do
   R=1; [ $W = imix ] && R=4
   XSKNF_GPU_LIB=$PWD/$L/libxsknf_gpu.so timeout -k 10 100 python tools/tune.py --workload $W --rotate $R --bpc 4 --rounds 5 2>>gpurun_out/abtp/err | sed "s|^{|{\"lib\": \"$L\", |" >> gpurun_out/abtp/res.jsonl || exit 1
  done
 done
done
cut -c1-160 gpurun_out/abtp/res.jsonl
