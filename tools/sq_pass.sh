#!/bin/bash
# SQ counters of one shape (tools/launch_n.py), run ON the GPU box:
#   tools/sq_pass.sh <tag> <workload> <shape>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/sq_$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES \
  --output-format csv -d "$OUT/a" -o run -- python3 "$R/tools/launch_n.py" --workload $2 --shape $3 --n 12 > "$OUT/a.log" 2>&1 \
  || { echo "pass a failed"; tail -5 "$OUT/a.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/b" -o run -- python3 "$R/tools/launch_n.py" --workload $2 --shape $3 --n 12 > "$OUT/b.log" 2>&1 \
  || { echo "pass b failed"; tail -5 "$OUT/b.log"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$OUT" xsknf_gpu
