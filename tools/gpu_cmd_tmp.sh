set -o pipefail
mkdir -p gpurun_out/nch
for rep in 1 2 3; do
for W in 1500 1024 800; do
  timeout -k 10 120 python tools/tune.py --workload $W --bpc 4 --rounds 5 --variants 16,3,2,0,18,1,24 >> gpurun_out/nch/res.jsonl 2>>gpurun_out/nch/err || exit 1
done; done
cut -c1-140 gpurun_out/nch/res.jsonl
