set -o pipefail
mkdir -p gpurun_out/r05h
for F in 4194304 13631488; do
  for L in lib llf; do
    LIB=$PWD/build/$L/libxsknf_gpu.so; [ $L = lib ] && LIB=$PWD/xsknf_amd/lib/libxsknf_gpu.so
    XSKNF_GPU_LIB=$LIB timeout -k 10 300 python tools/tune.py --workload 64 --frames $F --rotate 1 --rounds 5 --reps 5 2>>gpurun_out/r05h/err | sed "s|^{|{\"lib\": \"$L\", \"frames\": $F, |" >> gpurun_out/r05h/ab.jsonl || exit 1
  done
done
cat gpurun_out/r05h/ab.jsonl
