#!/bin/bash
# Cost of the checksummer's stores on top of the read footprints (GPU box).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$R/tools/build/hbm_probe
M=1048576
for wc in 0 1 16 32 64 128; do timeout -k 10 120 "$P" $M 2048 256 1504 20 $wc 1; done
for wc in 0 1 16 32 64; do timeout -k 10 120 "$P" $M 2048 256 64 20 $wc 1; done
for wc in 0 1 64; do timeout -k 10 120 "$P" $((M*9000/8192)) 8192 0 8192 20 $wc 1; done
