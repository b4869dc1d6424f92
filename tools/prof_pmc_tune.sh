#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc pass per group) over a short tune.py
# run of ONE launch shape, plus the same groups over the read probe (GPU box).
#   tools/prof_pmc_tune.sh <tag> <workload> <shape>
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; W=$2; S=$3
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
CGROUPS=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
)
i=0
for G in "${CGROUPS[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $G --output-format csv -d "$OUT/k$i" -o run \
    -- python3 "$R/tools/tune.py" --workload $W --variants $S --rounds 1 --reps 3 > "$OUT/k$i.json" 2> "$OUT/k$i.err"
  timeout -k 10 300 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -o run \
    -- "$R/tools/build/hbm_probe" 1048576 2048 256 1504 3 0 0 > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  i=$((i+1))
done
