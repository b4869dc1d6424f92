#!/bin/bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$R/tools/build/hbm_probe
M=1048576
export PROBE_HEAD=1
timeout -k 10 120 "$P" $M 2048 256 1504 8 0 0
