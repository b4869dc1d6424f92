#!/bin/bash
# Sector re-read vs side-buffer scatter (tools/hbm_probe PROBE_SIDE), plus the
# head-policy and store-shape probes, on the 1500 B and 64 B footprints (GPU box).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$R/tools/build/hbm_probe
M=1048576
PROBE_SIDE=1 timeout -k 10 120 "$P" $M 2048 256 1504 10 0 0
PROBE_SIDE=1 timeout -k 10 120 "$P" $M 2048 256 64 10 0 0
PROBE_SEQ=1 timeout -k 10 120 "$P" $M 2048 256 1504 10 0 0
PROBE_HEAD=1 timeout -k 10 120 "$P" $M 2048 256 1504 10 0 0
