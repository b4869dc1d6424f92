# Jumbo: deferred checks patched from the pooled kernel's patch list (mode 18) vs the scatter pass (run ON the GPU box).
set -o pipefail
for r in 1 2; do
timeout -k 10 300 python tools/tune.py --workload jumbo --bpc 4 --rounds 3 --reps 4 --variants 16,3,2,0,18,1,52 >> gpurun_out/jt.jsonl 2>>gpurun_out/jt.err || { tail gpurun_out/jt.err; exit 1; }
done
cut -c1-200 gpurun_out/jt.jsonl
