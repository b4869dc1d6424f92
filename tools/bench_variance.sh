# Three default bench.py runs back to back on one box (run ON the GPU box): run-to-run spread of the headline.
set -o pipefail
mkdir -p gpurun_out/var
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --secondary "" --cpu-seconds 0 > gpurun_out/var/b$i.json 2> gpurun_out/var/b$i.err || exit 1
done
for i in 1 2 3; do python3 -c "import json; d=json.load(open('gpurun_out/var/b$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
