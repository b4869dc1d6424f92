#!/bin/bash
# Read-bandwidth probe over the UMEM patterns of the BASELINE configs (GPU box).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$R/tools/build/hbm_probe
M=1048576
run() { timeout -k 10 120 "$P" "$@"; }
run $((M*1536/2048)) 2048 0 2048          # contiguous, 1.5 GiB
run $M 2048 256 1536                      # 1500B config footprint (16-B hull)
run $M 2048 0 1536                        # same bytes at chunk start
run $M 2048 256 2048                      # whole chunks, 2 GiB
run $M 1536 0 1536                        # packed 1536-B frames
run $M 4096 256 1536                      # libxdp default 4 KiB frames
run $M 2048 256 64                        # 64B config footprint
run $M 2048 256 128
run $((M*9000/2048)) 2048 0 2048          # ~ jumbo footprint contiguous
run $M 2048 256 1792
run $M 2048 0 1792
