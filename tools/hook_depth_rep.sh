set -o pipefail
B=tools/build/hook_bench
mkdir -p gpurun_out/hd2
for r in 1 2 3; do
 for cfg in "1500 64" "64 64" "1500 256"; do
  for D in 1 2; do
   timeout -k 10 30 $B async $cfg 2 ZEROCOPY $D >> gpurun_out/hd2/hook_depth_rep.jsonl 2>> gpurun_out/hd2/err || exit 1
  done
 done
done
cat gpurun_out/hd2/hook_depth_rep.jsonl
