#!/bin/bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$R/tools/build/hbm_probe
M=1048576
for wc in 0 1 -2 64 -64; do timeout -k 10 120 "$P" $M 2048 256 1504 20 $wc 0; done
for wc in 0 1 -2 -64; do timeout -k 10 120 "$P" $M 2048 256 64 20 $wc 0; done
