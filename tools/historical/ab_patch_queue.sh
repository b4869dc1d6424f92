#!/bin/bash
# A/B (needs build/ab_pq and build/tl_pq: a full A/B library and the product timeline
# build with -DXSKNF_PATCH_SHARED=1): one patch queue per block -- each wave
# publishes its finished units' lists, and waves whose streams are done patch
# any published unit of the block -- against each wave patching its own list
# after its last unit.  Hypothesis: the launch ends ~8 us after its last stream
# (the last wave's whole list); with the block's idle waves sharing the last
# units' patches it would end ~one unit's patches after it.  Parity first,
# then the two libraries interleaved (tools/tune.py), then timelines:
#   tools/ab_patch_queue.sh <tag>
set -o pipefail
TAG=${1:-patch_queue}
OUT=gpurun_out/ab
mkdir -p $OUT
XSKNF_GPU_LIB=$PWD/build/ab_pq/libxsknf_gpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_vs_reference.py \
  -k "full_size_configs or every_launch_shape or nic_offloaded or pool_units or device_batches or random_sweep" \
  > $OUT/${TAG}_parity.log 2>&1 || { tail -30 $OUT/${TAG}_parity.log; exit 1; }
tail -1 $OUT/${TAG}_parity.log
for rep in 1 2 3; do
  for L in xsknf_amd/lib build/ab_pq; do
    for W in 1500:1 1024:1 570:3 imix:3; do
      XSKNF_GPU_LIB=$PWD/$L/libxsknf_gpu.so timeout -k 10 200 python tools/tune.py --workload ${W%%:*} \
        --rotate ${W##*:} --rounds 7 2>/dev/null | sed "s|^{|{\"lib\": \"$L\", \"rep\": $rep, |" >> $OUT/${TAG}.jsonl || exit 1
    done
  done
done
for L in tl tl_pq; do
  for W in 1500:1 imix:3; do
    XSKNF_GPU_LIB=$PWD/build/$L/libxsknf_gpu.so timeout -k 10 200 python tools/timeline.py --workload ${W%%:*} \
      --rotate ${W##*:} | sed "s|^{|{\"lib\": \"$L\", |" >> $OUT/${TAG}_timeline.jsonl || exit 1
  done
done
python3 - $OUT/${TAG}.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["workload"], j["lib"])].append(j["us"])
for k in sorted(d): print(k, d[k])
PY
