#!/bin/bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$R/tools/build/hbm_probe
M=1048576
export PROBE_SEQ=1
timeout -k 10 120 "$P" $M 2048 256 1504 10 0 0
timeout -k 10 120 "$P" $M 2048 256 64 10 0 0
timeout -k 10 120 "$P" $((M*9000/8192)) 8192 0 8192 6 0 0
